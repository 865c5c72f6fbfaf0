// Device kernels of libsem_hip.so (included once, by sem_device.hip).
//
// Hot path (BASELINE.json north_star):
//   for every element e:  u_e = u[map[e]]                       (gather)
//                         d0 = D u_e,  d1 = u_e D^T              (D(x)I, I(x)D)
//                         w0 = G00 d0 + G01 d1, w1 = G01 d0 + G11 d1
//                         y_e = D^T w0 + w1 D                    (transposed pass)
//                         y[map[e]] += y_e                       (scatter-add)
// which equals the reference's per-element dense action
// einsum('pqrs,rs', Lse, u[loc]) (examples/poisson.py:168-193,
// examples/squirmer-axisymmetric.py:286) to rounding.
//
// CDNA4 mapping:
//  * GROUP = one wavefront's EPW = floor(64 / n) elements; lane = (element
//    slot k, line j).  Contractions along the lane's own column/row run in
//    registers with D as wave-uniform kernel arguments (SGPRs); the two
//    transposes go through a wave-private LDS tile.
//  * CHAIN = R rounds x 4 consecutive groups, processed by one 256-thread
//    workgroup (round by round, one group per wavefront).  Consecutive groups
//    of a chain usually share one column of nodes: the earlier group hands its
//    partial sums for that column to the later one through LDS ("carry"), so
//    every node has exactly one writer inside a chain and consecutive y rows
//    are completed by one workgroup (one XCD's L2), close in time.
//  * Chains are coloured at setup so that chains of one colour share no node;
//    one launch per colour.  Every packed map entry carries a 4-bit write code:
//    plain store for the first writer of a node in launch order,
//    read-modify-write for later writers, skip + register merge for a node
//    shared by the elements on two neighbouring lanes, carry-in for the node
//    handed over by the previous group, atomic only as a fallback.  No
//    atomics on structured (or any locality-ordered conforming) meshes.
//  * the map and the geometric factors are repacked at setup into
//    [group][row][lane] order: every wave-instruction streams one contiguous
//    run of HBM.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "sem_internal.h"

namespace semk {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;
// Groups per chain round = wavefronts per workgroup: 4.  At n = 17 the
// colour launches ran faster with 2-wave chains (p = 16 at 1e7 DOF: 0.165
// against 0.173 ms, profiles/r02/variants), but AUTO takes the seam plan
// there (one launch), on which 4-wave chains are ahead: 0.131
// against 0.136 ms (profiles/r02/final/chain_width).  SEM_CHAIN_WAVES
// (diagnostic builds) forces one value for every order.
#ifdef SEM_CHAIN_WAVES
constexpr int chain_waves_of(int) { return SEM_CHAIN_WAVES; }
#else
constexpr int chain_waves_of(int) { return 4; }
#endif
template <int N>
struct ChainWaves {
  static constexpr int value = chain_waves_of(N);
  static constexpr int block = value * WAVE;
};
constexpr int MAXN = 17;

// packed map entry = gid | code << CODE_SHIFT
constexpr int CODE_SHIFT = 28;
constexpr uint32_t GID_MASK = (1u << CODE_SHIFT) - 1u;
constexpr uint32_t W_STORE = 0;   // first writer: y = v   (y += v in accumulate mode)
constexpr uint32_t W_RMW = 1;     // later writer: y += v (no concurrent writer)
constexpr uint32_t W_SKIP = 2;    // value merged into another lane / padding
constexpr uint32_t W_ATOMIC = 3;  // fallback
constexpr uint32_t W_MERGE = 4;   // add the next lane's value before writing
constexpr uint32_t W_CARRY = 8;   // add the value handed over by the previous group
// SKIP | CARRY: row n-1 entry whose value the same lane adds to row 0 of its
// next round (block layout): not written by this round
constexpr uint32_t W_ROWCARRY = W_SKIP | W_CARRY;

#ifndef SEM_POISSON_MIN_WAVES
#define SEM_POISSON_MIN_WAVES 0  // 0: per-order choice (PoissonMinWaves)
#endif
#ifndef SEM_NT_MAP
#define SEM_NT_MAP 0  // map stream read with nontemporal loads
#endif
#ifndef SEM_NT_STORE
#define SEM_NT_STORE 1  // first-writer y stores nontemporal
#endif
#ifndef SEM_RMW_PREFETCH
#define SEM_RMW_PREFETCH 1  // Poisson: read read-modify-write targets before the last passes
#endif
// The prefetch holds n operands per lane through the last contractions:
// measured on MI355X at ~1e7 DOF it pays up to n = 13 (p = 12: 0.142 vs
// 0.163 ms) and costs at n = 17 (p = 16: 0.197 vs 0.176 ms; 246 vs 159
// VGPRs, profiles/r02/variants).
#ifndef SEM_RMW_PREFETCH_17
#define SEM_RMW_PREFETCH_17 0  // n = 17: 0 off, 1 / 2 as SEM_RMW_PREFETCH
#endif
template <int N>
struct RmwPrefetch {
  static constexpr int value = N <= 16 ? SEM_RMW_PREFETCH : SEM_RMW_PREFETCH_17;
};

// D1 in even-odd form.  D is centro-antisymmetric (D[N-1-i][N-1-j] =
// -D[i][j] on the symmetric GLL nodes), so with e_r = x_r + x_{N-1-r},
// o_r = x_r - x_{N-1-r} (r < H = N/2) both D x and D^T x need only
//   P[m][r] = (D[m][r] - D[m][N-1-r]) / 2,  Q[m][r] = (D[m][r] + D[m][N-1-r]) / 2
// plus, for odd N, the middle column cc[m] = D[m][H] and row rr[r] = D[H][r]:
// 2H^2 + 2H values instead of N^2 (40 vs 81 doubles at p = 8, so D fits the
// scalar register file next to the kernel's pointers) and ~40 % fewer FMAs.
// TR: the transposes PT[q][m] = P[m][q], QT[q][m] = Q[m][q] as well, for the
// device copy read with scalar loads (n >= SEM_D_SCALAR_LOAD_N): the D^T
// contractions then read each output row's 2H coefficients as two contiguous
// 8 x 8-byte runs (two s_load_dwordx16) instead of 2H strided single loads,
// each followed by a wait (the p = 12..16 stall)
#ifndef SEM_D_SCALAR_LOAD_N
#define SEM_D_SCALAR_LOAD_N 10
#endif
#ifndef SEM_DEO_TRANSPOSED
#define SEM_DEO_TRANSPOSED 1
#endif
template <int N>
struct DEOData {
  static constexpr int H = N / 2;
  static constexpr int C = N % 2;
  static constexpr bool TR = SEM_DEO_TRANSPOSED && N >= SEM_D_SCALAR_LOAD_N;
  double P[H * H];
  double Q[H * H];
  double cc[C ? H : 1];
  double rr[C ? H : 1];
  double PT[TR ? H * H : 1];
  double QT[TR ? H * H : 1];
};
// Q[m][q] and P[m][q] for a contraction over m at fixed q (D^T x)
#define DEO_QC(E, m, q) (DEOData<N>::TR ? (E)->QT[(q) * H + (m)] : (E)->Q[(m) * H + (q)])
#define DEO_PC(E, m, q) (DEOData<N>::TR ? (E)->PT[(q) * H + (m)] : (E)->P[(m) * H + (q)])

// How the kernels see D.  Up to n = 9 the even-odd halves are kernel
// arguments (SGPRs for the whole kernel).  Above, they no longer fit the
// 102-SGPR file and the compiler would spill them to VGPR lanes (two
// v_readlane per FMA operand); instead each contraction row re-reads its
// 2H values with scalar loads from a device copy: the pointer is laundered
// through an empty asm per row so the loads are neither hoisted nor CSE'd.
// (Round 3 tried a per-workgroup LDS copy read with broadcast ds_reads: no
// SGPR pressure, but every wave-wide read returns 64 copies of a value
// through the CU's LDS port -- slower at every order, p = 10 / 12 / 14 / 16:
// 0.131 / 0.137 / 0.153 / 0.158 against 0.122 / 0.131 / 0.138 / 0.138 ms,
// profiles/r03/high_order_d.)
template <int N>
using CDEOData = const __attribute__((address_space(4))) DEOData<N>;

template <int N, bool PTR = (N >= SEM_D_SCALAR_LOAD_N)>
struct DEO;

template <int N>
struct DEO<N, false> {
  DEOData<N> d;
  __device__ __forceinline__ const DEOData<N>* row() const { return &d; }
};

template <int N>
struct DEO<N, true> {
  const DEOData<N>* p;  // device copy (constant during the launch)
  __device__ __forceinline__ CDEOData<N>* row() const {
    CDEOData<N>* q = (CDEOData<N>*)(p);
    asm volatile("" : "+s"(q));
    return q;
  }
};

// D of the standard GLL basis as compile-time constants (csrc/deo_const.h,
// generated by tools/gen_deo_const.py from the library's own D): the
// coefficients become literal operands materialised by scalar moves where
// they are used, so they hold no registers across the round loop (the
// kernel-argument form keeps 80 SGPRs live and the allocator spills the
// excess to VGPR lanes, read back with v_readlane in every round).  Used
// only when the context's D equals the table bit for bit (sem_set_basis,
// DESIGN.md §4.1); any other basis runs the argument form.
template <int N>
struct DEOConstData {
  static constexpr bool available = false;
};
// SEM_CONST_D_PIN: each constant is materialised at its use (an empty asm on
// its SGPR pair), never hoisted out of the round loop
#ifndef SEM_CONST_D_PIN
#define SEM_CONST_D_PIN 0
#endif
}  // namespace semk
#include "deo_const.h"
namespace semk {
template <int N>
struct DEOConst {};  // tag: the contractions below read DEOConstData<N> at compile time

// compile-time loop: f(std::integral_constant<int, i>) for i = 0..K-1
template <class F, int... I>
__device__ __forceinline__ void sfor_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>()), ...);
}
template <int K, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_(f, std::make_integer_sequence<int, K>());
}

// the kernel's view of D: the constant table (CD) or the argument
template <int N, bool CD>
__device__ __forceinline__ auto deo_view(const DEO<N>& D) {
  if constexpr (CD)
    return DEOConst<N>();
  else
    return D;
}

// v = D x
template <int N, class DT>
__device__ __forceinline__ void deo_apply(const DT& D, const double (&x)[N],
                                          double (&v)[N]) {
  constexpr int H = N / 2;
  double e[H], o[H];
#pragma unroll
  for (int r = 0; r < H; ++r) {
    e[r] = x[r] + x[N - 1 - r];
    o[r] = x[r] - x[N - 1 - r];
  }
#pragma unroll
  for (int m = 0; m < H; ++m) {
    const auto E = D.row();
    double sp = 0.0, tp = 0.0;
    if constexpr (DEOData<N>::C) tp = E->cc[m] * x[H];
#pragma unroll
    for (int r = 0; r < H; ++r) {
      sp = fma(E->P[m * H + r], o[r], sp);
      tp = fma(E->Q[m * H + r], e[r], tp);
    }
    v[m] = sp + tp;
    v[N - 1 - m] = sp - tp;
  }
  if constexpr (DEOData<N>::C) {
    const auto E = D.row();
    double a = 0.0;
#pragma unroll
    for (int r = 0; r < H; ++r) a = fma(E->rr[r], o[r], a);
    v[H] = a;
  }
}

// v = D^T x  (the transpose is centro-antisymmetric with P^T <-> Q^T swapped)
template <int N, class DT>
__device__ __forceinline__ void deo_apply_t(const DT& D, const double (&x)[N],
                                            double (&v)[N]) {
  constexpr int H = N / 2;
  double e[H], o[H];
#pragma unroll
  for (int r = 0; r < H; ++r) {
    e[r] = x[r] + x[N - 1 - r];
    o[r] = x[r] - x[N - 1 - r];
  }
#pragma unroll
  for (int q = 0; q < H; ++q) {
    const auto E = D.row();
    double sp = 0.0, tp = 0.0;
    if constexpr (DEOData<N>::C) tp = E->rr[q] * x[H];
#pragma unroll
    for (int m = 0; m < H; ++m) {
      sp = fma(DEO_QC(E, m, q), o[m], sp);
      tp = fma(DEO_PC(E, m, q), e[m], tp);
    }
    v[q] = sp + tp;
    v[N - 1 - q] = sp - tp;
  }
  if constexpr (DEOData<N>::C) {
    const auto E = D.row();
    double a = 0.0;
#pragma unroll
    for (int m = 0; m < H; ++m) a = fma(E->cc[m], o[m], a);
    v[H] = a;
  }
}

// out[m] (m = 0..N-1) = (TR ? D^T x : D x), written to out[m * stride] pair by
// pair as the even-odd sums complete (a row pass stores into the lane's own
// LDS row): only e, o and one output pair are live, not the whole output
// column -- the register peak of the high-order column kernels
template <int N, bool TR, class DT>
__device__ __forceinline__ void deo_apply_to(const DT& D, const double (&x)[N], double* out) {
  constexpr int H = N / 2;
  double e[H], o[H];
#pragma unroll
  for (int r = 0; r < H; ++r) {
    e[r] = x[r] + x[N - 1 - r];
    o[r] = x[r] - x[N - 1 - r];
  }
#pragma unroll
  for (int m = 0; m < H; ++m) {
    const auto E = D.row();
    double sp = 0.0, tp = 0.0;
    if constexpr (DEOData<N>::C) tp = (TR ? E->rr[m] : E->cc[m]) * x[H];
#pragma unroll
    for (int r = 0; r < H; ++r) {
      sp = fma(TR ? DEO_QC(E, r, m) : E->P[m * H + r], o[r], sp);
      tp = fma(TR ? DEO_PC(E, r, m) : E->Q[m * H + r], e[r], tp);
    }
    out[m] = sp + tp;
    out[N - 1 - m] = sp - tp;
  }
  if constexpr (DEOData<N>::C) {
    const auto E = D.row();
    double a = 0.0;
#pragma unroll
    for (int r = 0; r < H; ++r) a = fma(TR ? E->cc[r] : E->rr[r], o[r], a);
    out[H] = a;
  }
}

// the same three contractions with D from the compile-time table: every
// coefficient is a constant expression (a literal operand where it is used)
template <int N>
__device__ __forceinline__ void deo_const_rows(const double (&x)[N], double (&e)[N / 2],
                                               double (&o)[N / 2]) {
#pragma unroll
  for (int r = 0; r < N / 2; ++r) {
    e[r] = x[r] + x[N - 1 - r];
    o[r] = x[r] - x[N - 1 - r];
  }
}
// TR false: out[m] = (D x)[m]; TR true: (D^T x)[m]; Store(m, value)
template <int N, bool TR, class Store>
__device__ __forceinline__ void deo_const_apply(const double (&x)[N], Store&& st) {
  using K = DEOConstData<N>;
  constexpr int H = N / 2;
  double e[H], o[H];
  deo_const_rows<N>(x, e, o);
  sfor<H>([&](auto mI) {
    constexpr int m = decltype(mI)::value;
    double sp = 0.0, tp = 0.0;
    if constexpr (N % 2) {
      double c = TR ? K::rr[m] : K::cc[m];
      if constexpr (SEM_CONST_D_PIN) asm volatile("" : "+s"(c));
      tp = c * x[H];
    }
    sfor<H>([&](auto rI) {
      constexpr int r = decltype(rI)::value;
      double a = TR ? K::Q[r * H + m] : K::P[m * H + r];
      double b = TR ? K::P[r * H + m] : K::Q[m * H + r];
      if constexpr (SEM_CONST_D_PIN) {  // materialised here, never hoisted
        asm volatile("" : "+s"(a));
        asm volatile("" : "+s"(b));
      }
      sp = fma(a, o[r], sp);
      tp = fma(b, e[r], tp);
    });
    st(m, sp + tp);
    st(N - 1 - m, sp - tp);
  });
  if constexpr (N % 2) {
    double a = 0.0;
    sfor<H>([&](auto rI) {
      constexpr int r = decltype(rI)::value;
      double c = TR ? K::cc[r] : K::rr[r];
      if constexpr (SEM_CONST_D_PIN) asm volatile("" : "+s"(c));
      a = fma(c, o[r], a);
    });
    st(H, a);
  }
}
template <int N>
__device__ __forceinline__ void deo_apply(const DEOConst<N>&, const double (&x)[N],
                                          double (&v)[N]) {
  deo_const_apply<N, false>(x, [&](int m, double t) { v[m] = t; });
}
template <int N>
__device__ __forceinline__ void deo_apply_t(const DEOConst<N>&, const double (&x)[N],
                                            double (&v)[N]) {
  deo_const_apply<N, true>(x, [&](int m, double t) { v[m] = t; });
}
template <int N, bool TR>
__device__ __forceinline__ void deo_apply_to(const DEOConst<N>&, const double (&x)[N],
                                             double* out) {
  deo_const_apply<N, TR>(x, [&](int m, double t) { out[m] = t; });
}

template <int N>
struct WVec {  // 1-D GLL quadrature weights
  double v[N];
};

// w[j] for a lane-varying j without dynamic indexing of the kernel arguments
template <int N>
__device__ __forceinline__ double pick(const WVec<N>& w, int j) {
  double r = w.v[0];
#pragma unroll
  for (int q = 1; q < N; ++q) r = (j == q) ? w.v[q] : r;
  return r;
}

// Ordering point for LDS traffic between lanes of ONE wavefront (a wave's LDS
// operations complete in issue order; this only stops the compiler moving
// them across the exchange).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void atomic_add_f64(double* p, double v) {
  unsafeAtomicAdd(p, v);  // global_atomic_add_f64, no return
}

// Read-modify-write targets were written earlier by this workgroup or by an
// earlier launch: read them past the CU's vector L1 (nt) so a line cached
// before the workgroup's own store is never reused.
__device__ __forceinline__ double rmw_load(const double* p) { return __builtin_nontemporal_load(p); }

// NT: nontemporal first-writer stores (the column kernels' row-contiguous
// scatter; the MFMA kernel's scattered 16 x 16 layout measured 10 % slower
// with them at p = 12)
template <bool NT = (SEM_NT_STORE != 0)>
__device__ __forceinline__ void emit1(double* __restrict__ y, uint32_t raw, double v,
                                      int accumulate) {
  const uint32_t a = (raw >> CODE_SHIFT) & 3u;
  double* dst = y + (raw & GID_MASK);
  if (a == W_STORE) {
    if constexpr (NT)
      __builtin_nontemporal_store(accumulate ? rmw_load(dst) + v : v, dst);
    else
      *dst = accumulate ? rmw_load(dst) + v : v;
  } else if (a == W_RMW) {
    *dst = rmw_load(dst) + v;
  } else if (a == W_ATOMIC) {
    atomic_add_f64(dst, v);
  }
}

// Poisson scatter with the read-modify-write operands already in registers
// (rmw_prefetch): no memory latency between the last contraction and the
// stores.  Safe because a RMW target's earlier writers are an earlier launch
// (colour), an earlier round of this chain (ended by a workgroup barrier) or
// an earlier operator in stream order -- never a concurrent wave.
// buffer-instruction cache policies (gfx950): nt = 2, sc1 = 16
constexpr int CPOL_NT = 2;

// y as a buffer resource: node ids are < 2^28, so byte offsets stay below
// the 2^31-byte range, and an offset of 2^31 reads 0 with no memory traffic
__device__ __forceinline__ __amdgpu_buffer_rsrc_t y_rsrc(const double* y) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(y), 0, 0x80000000, 0x00020000);
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int N, int AUX = CPOL_NT>
__device__ __forceinline__ void rmw_prefetch(const double* __restrict__ y,
                                             const uint32_t (&raw)[N], int accumulate,
                                             double (&prev)[N]) {
  // predicated without branches: a lane that needs no operand reads past the
  // end of the buffer range (returns 0, no memory traffic)
  const __amdgpu_buffer_rsrc_t ry = y_rsrc(y);
#pragma unroll
  for (int p = 0; p < N; ++p) {
    const uint32_t a = (raw[p] >> CODE_SHIFT) & 3u;
    const bool need = a == W_RMW || (a == W_STORE && accumulate);
    const uint32_t off = need ? (raw[p] & GID_MASK) * 8u : 0x80000000u;
    prev[p] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(ry, off, 0, AUX));
  }
}

__device__ __forceinline__ void emit1p(double* __restrict__ y, uint32_t raw, double v, double prev) {
  const uint32_t a = (raw >> CODE_SHIFT) & 3u;
  double* dst = y + (raw & GID_MASK);
  if (a == W_STORE || a == W_RMW) {  // prev = 0 for a first writer in overwrite mode
#if SEM_NT_STORE
      __builtin_nontemporal_store(prev + v, dst);
#else
      *dst = prev + v;
#endif
  } else if (a == W_ATOMIC) {
    atomic_add_f64(dst, v);
  }
}

// read-modify-write prefetch policy of a chain kernel: colour launches
// prefetch the operands, the seam plan has none (no read-modify-writes
// between chains)
struct NoWait {
  static constexpr int aux = CPOL_NT;
  static constexpr bool prefetch = true;
  __device__ void operator()() const {}
};
struct NoPrefetch {
  static constexpr int aux = CPOL_NT;
  static constexpr bool prefetch = false;
  __device__ void operator()() const {}
};

// Seam plan: a node written by several chains is not
// read-modified-written in colour order; each chain stores its partial sum
// in the node's slot for the chain's colour, buf[colour * n_node + gid], and
// a second launch (k_seam_sum) adds the slots into y in colour order.  All
// chains then run in one launch with no ordering and no read-modify-writes
// between chains.  The code action 3 (W_ATOMIC) means "seam slot" in this
// plan (the plan has no atomic chains).
struct SeamOut {
  double* base = nullptr;  // buf + colour * n_node * dpn of the chain
};
#ifndef SEM_NT_STORE_SEAM
#define SEM_NT_STORE_SEAM 1  // the seam plan's y and slot stores nontemporal
#endif
template <bool NT = (SEM_NT_STORE_SEAM != 0)>
__device__ __forceinline__ void st_seam(double v, double* dst) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, dst);
  else
    *dst = v;
}
__device__ __forceinline__ void emit1_seam(double* __restrict__ y, uint32_t raw, double v,
                                           int accumulate, const SeamOut& so) {
  const uint32_t a = (raw >> CODE_SHIFT) & 3u;
  const uint32_t gid = raw & GID_MASK;
  double* dst = y + gid;
  if (a == W_STORE)
    st_seam(accumulate ? rmw_load(dst) + v : v, dst);
  else if (a == W_RMW)  // first touch of a SEM_NODE_PRIOR node
    st_seam(rmw_load(dst) + v, dst);
  else if (a == W_ATOMIC)
    st_seam(v, so.base + gid);
}

__device__ __forceinline__ void emit2(double* __restrict__ y, uint32_t raw, double v0, double v1,
                                      int accumulate) {
  const uint32_t a = (raw >> CODE_SHIFT) & 3u;
  double* dst = y + 2 * (int64_t)(raw & GID_MASK);
  if ((a == W_STORE && !accumulate)) {
    *reinterpret_cast<double2*>(dst) = make_double2(v0, v1);
  } else if (a == W_STORE || a == W_RMW) {
    const double o0 = rmw_load(dst), o1 = rmw_load(dst + 1);
    *reinterpret_cast<double2*>(dst) = make_double2(o0 + v0, o1 + v1);
  } else if (a == W_ATOMIC) {
    atomic_add_f64(dst, v0);
    atomic_add_f64(dst + 1, v1);
  }
}

// SEM_LDS_SPLIT: tile loads of the nodal kernel as single 8-byte LDS reads.
// The compiler pairs neighbouring reads into ds_read2_b64, which the MI355X
// LDS serves at half the rate of two ds_read_b64 (MI355X_MICROARCH.md §LDS:
// 8 cycles against 2 x 2); a volatile access is never paired (and keeps the
// LDS address space: a generic volatile pointer became flat loads and
// spilled).  p = 8 at 1024^2, alternating on one box: 0.6726-0.6803 against
// 0.6827-0.6882 ms per step (profiles/r03/lds_split/).
#ifndef SEM_LDS_SPLIT
#define SEM_LDS_SPLIT 1
#endif
// the same for the column reads of the stored-factor kernel, from order
// SEM_LDS_SPLIT_STORED_N (profiles/r03/lds_split/stored/: p = 16 0.141-0.146
// -> 0.138-0.139 ms, but p = 6 0.126 -> 0.134 and p = 12 neutral)
#ifndef SEM_LDS_SPLIT_STORED_N
#define SEM_LDS_SPLIT_STORED_N 17
#endif
#ifndef SEM_LDS_SPLIT_AXI  // and of the fields-first axisymmetric nodal kernel
#define SEM_LDS_SPLIT_AXI 0
#endif
template <bool SPLIT>
__device__ __forceinline__ double lds_ld(const double* p) {
  if constexpr (SPLIT)
    return *(const volatile __attribute__((address_space(3))) double*)(p);
  else
    return *p;
}

// row i of the tile (RL doubles at row stride RS; 16-B aligned loads when
// both are even) -> registers
template <int N, int RS, int RL = RS, bool SPLIT = false>
__device__ __forceinline__ void load_row(const double* L, int i, double (&r)[RL]) {
  if constexpr (RL % 2 == 0 && RS % 2 == 0) {
    const double2* row = reinterpret_cast<const double2*>(L + i * RS);
#pragma unroll
    for (int s = 0; s < RL / 2; ++s) {
      const double2 v = row[s];
      r[2 * s] = v.x;
      r[2 * s + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int s = 0; s < RL; ++s) r[s] = lds_ld<SPLIT>(L + i * RS + s);
  }
}

// ACTIVE false: the lane stores at L + JUNK instead of its row (padding
// lanes of the wave-linear tile, whose row would run into the next tile row;
// an address select, not a branch: a masked store region spilled registers)
template <int N, int RS, int JUNK = 0>
__device__ __forceinline__ void store_row(double* L, int i, const double (&t)[N],
                                          bool active = true) {
  double* row = L + (active ? i * RS : JUNK);
  if constexpr (RS % 2 == 0) {
    double2* row2 = reinterpret_cast<double2*>(row);
#pragma unroll
    for (int s = 0; s < N / 2; ++s) row2[s] = make_double2(t[2 * s], t[2 * s + 1]);
    if (N % 2) row[N - 1] = t[N - 1];
  } else {
#pragma unroll
    for (int s = 0; s < N; ++s) row[s] = t[s];
  }
}

// LDS tiles: one N x RS slot per element of a group; the padding lanes
// (lane >= LW when N does not divide 64) of every wave share one scratch
// slot whose contents are never used.
// PAD: rows padded to 16 B for ds_read_b128 (odd N); p = 8 measured padded
// vs unpadded: 0.704 vs 0.720 ms (nodal).  At N = 9, slot stride 90 doubles
// and row stride 10 keep column and row accesses within 1.5x of conflict-free
// (bank model of MI355X_MICROARCH.md §LDS).
#ifndef SEM_TILE_PAD_STORED
#define SEM_TILE_PAD_STORED 1
#endif
// per order: p = 14 (n = 15) unpadded, 0.1209-0.1211 against 0.1234-0.1248
// ms per action (profiles/r04/knobs_high/, call P; p = 12 / 16 unchanged);
// p = 10 (n = 11) unpadded 0.1075-0.1085 against 0.1091-0.1094 (call S)
constexpr bool stored_pad(int n) { return SEM_TILE_PAD_STORED && n != 15 && n != 11; }
#ifndef SEM_TILE_PAD_NODAL
#define SEM_TILE_PAD_NODAL 0
#endif
#ifndef SEM_NODAL_EARLY_U
#define SEM_NODAL_EARLY_U 0
#endif
template <int N, bool PAD = true>
struct Tile {
  static constexpr int EPW = WAVE / N;
  static constexpr int LW = EPW * N;
  static constexpr int RS = (PAD && N % 2) ? N + 1 : N;  // PAD: 16-B aligned rows
  static constexpr int ES = N * RS;
  static constexpr int CW = ChainWaves<N>::value;
  static constexpr int TILE_SLOTS = CW * EPW + (LW < WAVE ? 1 : 0);
  __device__ static int slot(int wave, int k, bool in_wave) {
    return in_wave ? wave * EPW + k : CW * EPW;
  }
};

// Wave-linear tiles (nodal Poisson kernel): the wave's EPW element tiles
// side by side, element k at column offset k*N of one N x WL_RS array,
//   T[k][r][c] at  wave base + r*WL_RS + k*N + c,   WL_RS = 65 (= 1 mod 32).
// A column access (fixed r) is the wave's lanes in order, a row access
// (lane (k, j) reads row j) is lane + 64 j + c: both free of bank conflicts
// for 64-bit LDS accesses (MI355X_MICROARCH.md §LDS), where the element-slot
// layout (slot stride N*N) has 2-way conflicts on every column access.  The
// padding lanes' columns are the spare columns LW..64 of each row; their
// row stores go to a junk row after the wave's N rows (theirs would run into
// the next tile row).
#ifndef SEM_TILE_WL
#define SEM_TILE_WL 0
#endif
constexpr int WL_RS = 65;
template <int N>
struct WLTile {
  static constexpr int RS = WL_RS;
  static constexpr int LW = (WAVE / N) * N;
  static constexpr int WS = N * WL_RS + N;  // doubles per wave: N rows + the junk row
  static constexpr int JUNK = N * WL_RS - LW;  // junk row, from a padding lane's base
  __device__ static int base(int wave, int k) { return wave * WS + k * N; }
};



// Row pass on a wave-private tile: the lane's row j (written column-wise by
// the wave and synchronised) is contracted with D (or D^T when TR) and
// written back, so the tile again holds the result in column layout.  REL
// differentiates relative to the row's first entry (see poisson_group_nodal).
// RL: doubles loaded per row (RS, or N on the wave-linear tile); ACTIVE:
// whether the lane stores its row.
#ifndef SEM_ROW_STORE_PAIRS_N
#define SEM_ROW_STORE_PAIRS_N 17  // orders from which row passes store output pairs directly
#endif
// the stored-factor kernel's tile: wave-linear from order
// SEM_TILE_WL_STORED_N (conflict-free column and row accesses, §4.6; rows
// of 8-byte reads instead of 16-byte pairs), below the orders whose row
// passes store output pairs directly (their padding lanes have no junk row)
#ifndef SEM_TILE_WL_STORED_N
#define SEM_TILE_WL_STORED_N 99
#endif
template <int N>
struct StoredTile {
  static constexpr bool wl = N >= SEM_TILE_WL_STORED_N && N < SEM_ROW_STORE_PAIRS_N;
  static constexpr int RS = wl ? WL_RS : Tile<N, stored_pad(N)>::RS;
  static constexpr int RL = wl ? N : RS;  // doubles loaded per row
  static constexpr int JUNK = wl ? WLTile<N>::JUNK : 0;
};
template <int N, int RS, bool TR, bool REL, int RL = RS, int JUNK = 0, bool SPLIT = false,
          class DT = DEO<N>>
__device__ __forceinline__ void row_pass(double* L, int j, const DT& D, bool active = true) {
  double r[RL], x[N];
  load_row<N, RS, RL, SPLIT>(L, j, r);
#pragma unroll
  for (int q = 0; q < N; ++q) x[q] = REL ? r[q] - r[0] : r[q];
  if constexpr (N >= SEM_ROW_STORE_PAIRS_N) {
    // the lane rewrites only its own row: no ordering point needed between
    // its loads and its stores (the compiler orders them by address)
    deo_apply_to<N, TR>(D, x, L + j * RS);
  } else {
    double t[N];
    if constexpr (TR)
      deo_apply_t<N>(D, x, t);
    else
      deo_apply<N>(D, x, t);
    wave_sync();
    store_row<N, RS, JUNK>(L, j, t, active);
  }
  wave_sync();
}

// The coded map of group g, row by row, as raw 32-bit entries gid | code << 28.
// M16: the packed map holds 16-bit entries (gid - base) | code << 12 with one
// 32-bit base per group row (a row of a group spans < 4096 node ids on a
// locality-ordered mesh: 57 consecutive ids at p = 8 on the structured
// mesh), read with scalar loads -- 2 B instead of 4 per element node.  A
// group with a wider row (e.g. one that wraps into the next element column)
// is flagged and reads the 32-bit map instead (uniform branch per wave).
// Pattern table (the PAT kernels, sem_ctx::map_pat): groups whose 16-bit
// entries (offsets and codes) are the same share one copy -- on a structured
// numbering every row's offsets are the same run and the codes follow a few
// layouts -- so p16 holds [pattern][r][lane] and the group's pattern id sits
// in bits 28-31 of its bases 1..4 (node ids are < 2^28): the per-group map
// stream shrinks to the N bases.
struct MapRef {
  const uint32_t* __restrict__ p32;  // [slot][r][lane] gid | code << 28
  const uint16_t* __restrict__ p16;  // [slot][r][lane] (gid - base) | code << 12
  const uint32_t* __restrict__ base;  // [slot][r]
};
constexpr uint32_t M16_OFF_MASK = 0xFFFu;
constexpr uint32_t M16_WIDE = 0xFFFFFFFFu;  // base[slot][0]: this group uses the 32-bit map
constexpr int M16_CODE_SHIFT = 12;

// orders with pattern-table (PAT) kernels (SEM_MAP_PATTERN_N, a bit per n;
// the host builds a table only for these): every order from n = 3 --
// measured faster at p = 4 / 6 / 8 / 10 / 12 / 14 / 16.  The
// pattern id sits in the top 4 bits of bases 1..id_rows (min(4, n - 1)):
// up to 16^id_rows patterns.
#ifndef SEM_MAP_PATTERN_N
#define SEM_MAP_PATTERN_N 0x3FFF8u
#endif
template <int N>
struct PatternMap {
  static constexpr bool value = N >= 3 && ((SEM_MAP_PATTERN_N >> N) & 1u);
  static constexpr int id_rows = N - 1 < 4 ? N - 1 : 4;
};

template <int N, bool M16 = false, bool LD = false, bool PAT = false>
__device__ __forceinline__ void load_map(const MapRef& m, int64_t g, int lane, bool in_wave,
                                         uint32_t (&raw)[N]) {
  constexpr int LW = Tile<N>::LW;
  bool wide = !M16;
  if constexpr (M16) {
    // offsets and bases are issued together, ahead of the (rare, uniform)
    // wide-group branch: a branch on the base before the offset loads
    // serialised two memory latencies and measured 8 % slower
    // padding lanes load a valid entry (lane clamped) and discard it: no
    // load under a branch
    const uint32_t* bp = m.base + g * N;  // g is wave-uniform: scalar loads
    uint32_t o[N], b[N];
    if constexpr (PAT) {  // the pattern's entries follow the bases
#pragma unroll
      for (int r = 0; r < N; ++r) b[r] = bp[r];
      constexpr int Q = PatternMap<N>::id_rows;
      int64_t pid = 0;
#pragma unroll
      for (int q = 1; q <= Q; ++q) pid |= (int64_t)(b[q] >> 28) << (4 * (q - 1));
      const uint16_t* mp = m.p16 + pid * (int64_t)(N * LW) + (in_wave ? lane : LW - 1);
#pragma unroll
      for (int r = 0; r < N; ++r) {
        const uint32_t t = mp[r * LW];
        o[r] = in_wave ? t : (W_SKIP << M16_CODE_SHIFT);
      }
    } else {
      const uint16_t* mp = m.p16 + g * (int64_t)(N * LW) + (in_wave ? lane : LW - 1);
#pragma unroll
      for (int r = 0; r < N; ++r) {
        const uint32_t t = mp[r * LW];
        o[r] = in_wave ? t : (W_SKIP << M16_CODE_SHIFT);
      }
#pragma unroll
      for (int r = 0; r < N; ++r) b[r] = bp[r];
    }
    if constexpr (PAT)  // bases 1..Q carry the pattern id above the node id
#pragma unroll
      for (int r = 1; r <= PatternMap<N>::id_rows; ++r) b[r] &= GID_MASK;
#pragma unroll
    for (int r = 0; r < N; ++r)
      raw[r] = (b[r] + (o[r] & M16_OFF_MASK)) | ((o[r] >> M16_CODE_SHIFT) << CODE_SHIFT);
    wide = b[0] == M16_WIDE;
  }
  if (wide) {  // 32-bit map (M16: a group whose rows span >= 4096 ids)
    // LD (RawLaunder): the rare wide group's per-lane offset is re-formed
    // here, so the compiler cannot hoist p32 + lane out of the round loop as
    // a 64-bit VGPR address (spilled to scratch at the headline's register
    // limit, one store and one reload per round)
    if constexpr (M16 && LD) asm volatile("" : "+v"(lane));
    const uint32_t* mp = m.p32 + g * (int64_t)(N * LW) + lane;
#pragma unroll
    for (int r = 0; r < N; ++r)
#if SEM_NT_MAP
      raw[r] = in_wave ? __builtin_nontemporal_load(mp + r * LW) : (W_SKIP << CODE_SHIFT);
#else
      raw[r] = in_wave ? mp[r * LW] : (W_SKIP << CODE_SHIFT);
#endif
  }
}

// Next-round map prefetch into the caches (SEM_MAP_TOUCH, column kernel with
// the 16-bit map): the 16-bit entries of group g (N * LW * 2 bytes) and its
// N bases, read as dwords by the wave's lanes -- no registers are held for
// the data, only the loaded dwords until MapTouch::done, which an empty asm
// consumes at the end of the round (a load whose value is unused would be
// dropped; consuming it earlier would wait for it).  The next round's
// load_map then finds its lines in L2.
#ifndef SEM_MAP_TOUCH
#define SEM_MAP_TOUCH 0
#endif
template <int N>
struct MapTouch {
  static constexpr int LW = Tile<N>::LW;
  static constexpr int DW = (N * LW * 2 + 3) / 4;  // dwords of 16-bit entries
  static constexpr int K = (DW + WAVE - 1) / WAVE;
  uint32_t t[K + 1];
  __device__ __forceinline__ void issue(const MapRef& m, int64_t g, int lane) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(m.p16 + g * (int64_t)(N * LW));
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int d = k * WAVE + lane;
      t[k] = p[d < DW ? d : DW - 1];
    }
    t[K] = m.base[g * N + (lane < N ? lane : N - 1)];
  }
  __device__ __forceinline__ void done() {
#pragma unroll
    for (int k = 0; k <= K; ++k) asm volatile("" ::"v"(t[k]));
  }
};

// ---------------------------------------------------------------------------
// One group of the Poisson action with STORED factors: returns y_e[p][j]
// (p = 0..N-1) of the lane's column j in v[], and the raw coded map entries.
//   mapP[g][r][k*N + j] = map[e][r][j] | code,  GP[g][c][r][k*N + j] = G_c(e; r, j)
// ---------------------------------------------------------------------------
template <int N, bool M16, class Pre = NoWait, bool LD = false, bool PAT = false,
          class DT = DEO<N>>
__device__ __forceinline__ void poisson_group_stored(const MapRef& mref,
                                                     const double* __restrict__ GP,
                                                     const double* __restrict__ u, int64_t g,
                                                     int lane, int j, bool in_wave, double* L,
                                                     const DT& D, uint32_t (&raw)[N],
                                                     double (&v)[N], const double* __restrict__ y,
                                                     int accumulate, double (&prev)[N],
                                                     const Pre& pre = Pre()) {
  using T = Tile<N, stored_pad(N)>;
  constexpr int LW = T::LW;
  constexpr int RS = StoredTile<N>::RS;
  constexpr int RL = StoredTile<N>::RL;
  constexpr int JUNK = StoredTile<N>::JUNK;
  const bool act = in_wave || !StoredTile<N>::wl;
  constexpr bool SP = N >= SEM_LDS_SPLIT_STORED_N;
  const double* gp = GP + g * (int64_t)(3 * N * LW) + lane;
  double uc[N];
  load_map<N, M16, LD, PAT>(mref, g, lane, in_wave, raw);
#pragma unroll
  for (int r = 0; r < N; ++r) {
    uc[r] = u[raw[r] & GID_MASK];
  }
  // column j: d0[m][j] = sum_r D[m][r] u[r][j]     (TensorProduct.deriv dim 0)
  double d0[N];
  deo_apply<N>(D, uc, d0);
#pragma unroll
  for (int r = 0; r < N; ++r) L[r * RS + j] = uc[r];
  wave_sync();
  // row i = j: d1[i][q] = sum_s D[q][s] u[i][s]     (TensorProduct.deriv dim 1)
  row_pass<N, RS, false, false, RL, JUNK>(L, j, D, act);
  // column j: w0/w1, and ya = D^T w0 along xi0 (kept in v); w1 -> tile
  {
    double w0[N];
#pragma unroll
    for (int m = 0; m < N; ++m) {
      const double d1 = lds_ld<SP>(L + m * RS + j);
      const double g00 = gp[(0 * N + m) * LW];
      const double g01 = gp[(1 * N + m) * LW];
      const double g11 = gp[(2 * N + m) * LW];
      w0[m] = fma(g00, d0[m], g01 * d1);
      L[m * RS + j] = fma(g01, d0[m], g11 * d1);  // w1, same lane's slot
    }
    constexpr int PF = Pre::prefetch ? RmwPrefetch<N>::value : 0;
    if constexpr (PF) pre();
    if constexpr (PF == 1) rmw_prefetch<N, Pre::aux>(y, raw, accumulate, prev);
    deo_apply_t<N>(D, w0, v);
    if constexpr (PF == 2) rmw_prefetch<N, Pre::aux>(y, raw, accumulate, prev);
  }
  wave_sync();
  // row i = j: yb[i][q] = sum_n D[n][q] w1[i][n]
  row_pass<N, RS, true, false, RL, JUNK>(L, j, D, act);
#pragma unroll
  for (int p = 0; p < N; ++p) v[p] += lds_ld<SP>(L + p * RS + j);
  wave_sync();  // the tile is rewritten by the next group of this wave
}

// 1/x to full double precision without the IEEE division sequence:
// hardware reciprocal + two Newton steps (x is a Jacobian determinant, far
// from 0 and from the denormal range once sem_geom_from_nodes accepted it).
__device__ __forceinline__ double fast_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// ---------------------------------------------------------------------------
// One group of the Poisson action with NODAL geometry: the factors of the
// lane's column are re-derived from the GLL node coordinates XG[gid] =
// x_phys, the reference's own per-element order of work (sem/discrete.py:
// 189-209 -> sem/mapping.py:105-119 -> sem/linalg.py:105-115, detJxW
// sem/discrete.py:594-597):
//   J = [[dx/dr, dx/ds], [dy/dr, dy/ds]] (r = xi0 along the column, s = xi1),
//   G00 = W (J11^2 + J01^2)/det, G01 = -W (J11 J10 + J01 J00)/det,
//   G11 = W (J10^2 + J00^2)/det,   W = w_m w_j,
// i.e. detJxW * invJ invJ^T.  Every line of coordinates is differentiated
// relative to its first node (D annihilates constants), so O(1) coordinates
// do not cancel against O(h) differences.  Tiles: A (x, then u, then w1)
// and B (y).  Measured at p = 8: this order (factors first, x and y
// transposed together) beats the fully fused order (u/x/y/w1 one tile pass
// each, no factor arrays): 0.684 vs 0.714 ms.
// ---------------------------------------------------------------------------

template <int N>
__device__ __forceinline__ void gather_x(const double2* __restrict__ XG, const uint32_t (&raw)[N],
                                         int j, double2 (&xc)[N]) {
#pragma unroll
  for (int r = 0; r < N; ++r) {
    xc[r] = XG[raw[r] & GID_MASK];
  }
}

template <int N>
__device__ __forceinline__ void gather_u(const double* __restrict__ u, const uint32_t (&raw)[N],
                                         double (&uc)[N]) {
#pragma unroll
  for (int r = 0; r < N; ++r) {
    uc[r] = u[raw[r] & GID_MASK];
  }
}

// geometry of the group from its node coordinates: (dx/dr, dy/dr) along the
// column, (dx/ds, dy/ds) along the row -> G00, G01 in registers, G11 parked
// in tile B (free until the next group) to save registers
// the nodal kernel's tile: wave-linear (SEM_TILE_WL) below the orders whose
// row passes store pairs directly (unmasked), element slots otherwise
template <int N>
struct NodalTile {
  static constexpr bool wl = SEM_TILE_WL && N < SEM_ROW_STORE_PAIRS_N;
  static constexpr int RS = wl ? WL_RS : Tile<N, SEM_TILE_PAD_NODAL>::RS;
  static constexpr int RL = wl ? N : RS;  // doubles loaded per row
  static constexpr int JUNK = wl ? WLTile<N>::JUNK : 0;
  static constexpr bool split = SEM_LDS_SPLIT;
};

// SEM_W_SCALAR_LOAD: the nodal geometry reads w_m with scalar loads from the
// device copy once per round (pointer laundered, so neither hoisted nor kept)
// instead of holding the 2n SGPRs of the kernel argument for the whole launch
#ifndef SEM_W_SCALAR_LOAD
#define SEM_W_SCALAR_LOAD 0
#endif
using CWPtr = const __attribute__((address_space(4))) double*;
__device__ __forceinline__ CWPtr wrow(const double* wp) {
  CWPtr q = (CWPtr)wp;
  if constexpr (SEM_W_SCALAR_LOAD) asm volatile("" : "+s"(q));
  return q;
}
template <int N>
__device__ __forceinline__ double wsel(const WVec<N>& w, CWPtr q, int m) {
  if constexpr (SEM_W_SCALAR_LOAD)
    return q[m];
  else
    return w.v[m];
}
template <int N, class DT>
__device__ __forceinline__ void nodal_geometry(const double2 (&xc)[N], int j, double* A, double* B,
                                               const DT& D, const WVec<N>& w, double wj,
                                               double (&g00)[N], double (&g01)[N], bool in_wave, const double* wp = nullptr) {
  constexpr int RS = NodalTile<N>::RS;
  constexpr int RL = NodalTile<N>::RL;
  double jr0[N], jr1[N];
  {
    double ta[N], tb[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
      ta[r] = xc[r].x - xc[0].x;
      tb[r] = xc[r].y - xc[0].y;
    }
    deo_apply<N>(D, ta, jr0);
    deo_apply<N>(D, tb, jr1);
  }
#pragma unroll
  for (int r = 0; r < N; ++r) {
    A[r * RS + j] = xc[r].x;
    B[r * RS + j] = xc[r].y;
  }
  wave_sync();
  {
    double xa[RL], xb[RL], ra[N], rb[N], ta[N], tb[N];
    load_row<N, RS, RL, NodalTile<N>::split>(A, j, xa);
    load_row<N, RS, RL, NodalTile<N>::split>(B, j, xb);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      ra[q] = xa[q] - xa[0];
      rb[q] = xb[q] - xb[0];
    }
    deo_apply<N>(D, ra, ta);
    deo_apply<N>(D, rb, tb);
    wave_sync();
    store_row<N, RS, NodalTile<N>::JUNK>(A, j, ta, in_wave || !NodalTile<N>::wl);
    store_row<N, RS, NodalTile<N>::JUNK>(B, j, tb, in_wave || !NodalTile<N>::wl);
  }
  wave_sync();
  const auto wq = wrow(wp);
#pragma unroll
  for (int m = 0; m < N; ++m) {
    constexpr bool SP = NodalTile<N>::split;
    const double js0 = lds_ld<SP>(A + m * RS + j), js1 = lds_ld<SP>(B + m * RS + j);
    const double det = jr0[m] * js1 - js0 * jr1[m];
    // (w_m w_j) / det, associated so that no loop-invariant w_m w_j array
    // is hoisted out of the round loop (9 doubles spilled at 4 waves/SIMD)
    const double sc = wsel<N>(w, wq, m) * (wj * fast_rcp(det));
    g00[m] = sc * fma(js1, js1, js0 * js0);
    g01[m] = -sc * fma(js1, jr1[m], js0 * jr0[m]);
    B[m * RS + j] = sc * fma(jr1[m], jr1[m], jr0[m] * jr0[m]);  // G11, own slot
  }
  wave_sync();  // tile A is rewritten next
}

// the Laplacian of the group on tile A with G00/G01 in registers, G11 in B
template <int N, class Pre = NoWait, class DT = DEO<N>>
__device__ __forceinline__ void nodal_laplacian(const double (&uc)[N], int j, double* A,
                                                const double* B, const DT& D,
                                                const double (&g00)[N], const double (&g01)[N],
                                                double (&v)[N], const double* __restrict__ y,
                                                const uint32_t (&raw)[N], int accumulate,
                                                double (&prev)[N], bool in_wave,
                                                const Pre& pre = Pre()) {
  constexpr int RS = NodalTile<N>::RS;
  constexpr int RL = NodalTile<N>::RL;
  const bool act = in_wave || !NodalTile<N>::wl;
  double d0[N];
  deo_apply<N>(D, uc, d0);
#pragma unroll
  for (int r = 0; r < N; ++r) A[r * RS + j] = uc[r];
  wave_sync();
  constexpr bool SP = NodalTile<N>::split;
  row_pass<N, RS, false, false, RL, NodalTile<N>::JUNK, SP>(A, j, D, act);
  {
    double w0[N];
#pragma unroll
    for (int m = 0; m < N; ++m) {
      const double d1 = lds_ld<SP>(A + m * RS + j);
      w0[m] = fma(g00[m], d0[m], g01[m] * d1);
      A[m * RS + j] = fma(g01[m], d0[m], lds_ld<SP>(B + m * RS + j) * d1);
    }
    constexpr int PF = Pre::prefetch ? RmwPrefetch<N>::value : 0;
    if constexpr (PF) pre();
    if constexpr (PF == 1) rmw_prefetch<N, Pre::aux>(y, raw, accumulate, prev);
    deo_apply_t<N>(D, w0, v);
    if constexpr (PF == 2) rmw_prefetch<N, Pre::aux>(y, raw, accumulate, prev);
  }
  wave_sync();
  row_pass<N, RS, true, false, RL, NodalTile<N>::JUNK, SP>(A, j, D, act);
#pragma unroll
  for (int p = 0; p < N; ++p) v[p] += lds_ld<SP>(A + p * RS + j);
  wave_sync();  // the tiles are rewritten by the next group of this wave
}

// One group of the Poisson action with NODAL geometry (no prefetch).
template <int N, bool M16, class Pre = NoWait, bool LD = false, bool PAT = false,
          class DT = DEO<N>>
__device__ __forceinline__ void poisson_group_nodal(const MapRef& mref,
                                                    const double2* __restrict__ XG,
                                                    const double* __restrict__ u, int64_t g,
                                                    int lane, int j, bool in_wave, double* A,
                                                    double* B, const DT& D,
                                                    const WVec<N>& w, double wj,
                                                    uint32_t (&raw)[N], double (&v)[N],
                                                    const double* __restrict__ y, int accumulate,
                                                    double (&prev)[N], const Pre& pre = Pre(), const double* wp = nullptr) {
  double uc[N];
  double2 xc[N];
  load_map<N, M16, LD, PAT>(mref, g, lane, in_wave, raw);
  gather_x<N>(XG, raw, j, xc);
#if SEM_NODAL_EARLY_U
  gather_u<N>(u, raw, uc);
#endif
  double g00[N], g01[N];
  nodal_geometry<N>(xc, j, A, B, D, w, wj, g00, g01, in_wave, wp);
#if !SEM_NODAL_EARLY_U
  gather_u<N>(u, raw, uc);
#endif
  nodal_laplacian<N>(uc, j, A, B, D, g00, g01, v, y, raw, accumulate, prev, in_wave, pre);
}


// the value of lane + 1 (lane 63: its own).  SEM_DPP_SHIFT: a DPP
// wave_shl:1 move per dword (two VALU moves) instead of __shfl_down, whose
// ds_bpermute goes through the LDS and waits on it.  Below n = 17 only: at
// p = 16 the DPP form lifts the stored seam kernel to 169 VGPRs (2 waves per
// SIMD), and holding it at 3 waves with a launch bound changed its code for
// the worse -- 0.134 ms per action with __shfl_down against 0.152 (DPP,
// 3-wave bound) and 0.157 (DPP), profiles/r03/p16_regression/.
#ifndef SEM_DPP_SHIFT
#define SEM_DPP_SHIFT 1
#endif
#ifndef SEM_DPP_SHIFT_MAX_N
#define SEM_DPP_SHIFT_MAX_N 17
#endif
// DPP17: the DPP form at n = 17 as well (the constant-D kernels: 128 VGPRs
// either way there, 17 fewer LDS round trips per round; p = 16 0.1196-0.1226
// against 0.1225-0.1253 ms per action, profiles/r04/knobs_high/u_*)
template <int N, bool DPP17 = false>
__device__ __forceinline__ double lane_next(double x) {
  if constexpr (SEM_DPP_SHIFT && (N < SEM_DPP_SHIFT_MAX_N || DPP17)) {
    constexpr int WAVE_SHL1 = 0x130;
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, WAVE_SHL1, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(lo, lo, WAVE_SHL1, 0xF, 0xF, false));
  } else {
    return __shfl_down(x, 1, WAVE);
  }
}

#ifndef SEM_ROUND_SYNC_ALWAYS
#define SEM_ROUND_SYNC_ALWAYS 0
#endif
constexpr int CARRY_BUFS = 3;
#ifndef SEM_LANE_RECOMPUTE
#define SEM_LANE_RECOMPUTE 0
#endif

// Scatter of one group's column values through the coded map, with the
// in-group merge (next lane) and the chain carry (previous group) applied.
// ncomp values per node (1: Poisson, 2: axisymmetric block).
// DOT (seam plan, overwrite mode, one DOF per node): dot += u[gid] * value
// at every STORE -- the node's one and only final value outside the seams.
template <int N, int NC, bool PRE = false, int CW = ChainWaves<N>::value, bool SEAM = false,
          bool DOT = false, bool LD = false, bool DPP17 = false>
__device__ __forceinline__ void chain_emit(double* __restrict__ y, const uint32_t (&raw_in)[N],
                                           double (&v)[NC][N], int lane, int wave, int rd,
                                           bool in_wave, double (*carry)[CW][NC][N],
                                           double (&rowc)[NC], int accumulate, bool round_sync,
                                           const double* prev = nullptr,
                                           const SeamOut& so = SeamOut(),
                                           const double* __restrict__ du = nullptr,
                                           double* dot = nullptr) {
  constexpr int LW = Tile<N>::LW;
  uint32_t raw[N];
#pragma unroll
  for (int p = 0; p < N; ++p) {
    raw[p] = raw_in[p];
    // LD: the scatter recomputes its byte offsets from the coded map entries
    // (the compiler would otherwise keep the gather's offsets live through
    // the whole group next to the entries themselves: a scratch spill per
    // round at the headline's register limit)
    if constexpr (LD) asm volatile("" : "+v"(raw[p]));
  }
  // row carry between rounds (block layout): before any merge, row 0 takes
  // the row n-1 value this lane held back in the previous round
  const bool rc_out = (raw[N - 1] >> CODE_SHIFT) == W_ROWCARRY;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const double out = rc_out ? v[c][N - 1] : 0.0;
    v[c][0] += rowc[c];
    rowc[c] = out;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int p = 0; p < N; ++p) {
      const double vn = lane_next<N, DPP17>(v[c][p]);
      if ((raw[p] >> CODE_SHIFT) & W_MERGE) v[c][p] += vn;
    }
  // hand the last lane's column to the next group of the chain
  // SEM_LANE_RECOMPUTE: the lane tests are re-evaluated every round (the
  // lane id laundered) instead of kept as loop-invariant SGPR masks, which
  // the allocator spills to VGPR lanes at the register limit
  if constexpr (SEM_LANE_RECOMPUTE) asm volatile("" : "+v"(lane));
  if (lane == LW - 1) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int p = 0; p < N; ++p) carry[rd % CARRY_BUFS][wave][c][p] = v[c][p];
  }
  __syncthreads();
  if (lane == 0) {
    const double* src = (wave > 0) ? &carry[rd % CARRY_BUFS][wave - 1][0][0]
                                   : &carry[(rd + CARRY_BUFS - 1) % CARRY_BUFS][CW - 1][0][0];
#pragma unroll
    for (int p = 0; p < N; ++p)
      if ((raw[p] >> CODE_SHIFT) & W_CARRY) {
#pragma unroll
        for (int c = 0; c < NC; ++c) v[c][p] += src[c * N + p];
      }
  }
  if (in_wave) {
#pragma unroll
    for (int p = 0; p < N; ++p) {
      if constexpr (SEAM && NC == 1) {
        emit1_seam(y, raw[p], v[0][p], accumulate, so);
        if constexpr (DOT)
          if (((raw[p] >> CODE_SHIFT) & 3u) == W_STORE)
            *dot = fma(du[raw[p] & GID_MASK], v[0][p], *dot);
      }
      else if constexpr (PRE)
        emit1p(y, raw[p], v[0][p], prev[p]);
      else if (NC == 1)
        emit1(y, raw[p], v[0][p], accumulate);
      else if (SEAM && ((raw[p] >> CODE_SHIFT) & 3u) == W_ATOMIC)  // seam slot (2 DOFs)
        reinterpret_cast<double2*>(so.base)[raw[p] & GID_MASK] =
            make_double2(v[0][p], v[NC - 1][p]);
      else
        emit2(y, raw[p], v[0][p], v[NC - 1][p], accumulate);
    }
  }
  // this round's stores complete before the next round's read-modify-writes
  // of the same nodes: only plans in which a chain writes a node in two
  // rounds need it (SeamPlan::round_sync); the carry slots need no second
  // barrier with three buffers (a slot is rewritten three rounds later,
  // after its reader has passed the next round's first barrier)
  if (SEM_ROUND_SYNC_ALWAYS || round_sync) __syncthreads();
}

// Workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share
// one L2).  With SEM_XCD_SWIZZLE the chain index is remapped so that each XCD
// works on one contiguous run of chains (neighbouring chains share node
// columns of u / x_phys and the partial 128-B lines of y at their ends); a
// bijection of [0, nwg) for any nwg.  Measured on one MI355X
// (profiles/r04/xcd/, kernel median ms per action, swizzled / dealt): cfg2
// 256^2 (2,341 chains) 0.042 / 0.044; the headline 1024^2 (9,472) 0.623 -
// 0.630 / 0.619 with 0.08 GB less PMC fetch; p = 2 / 4 / 6 / 10 / 16 at 1e7
// DOF 2-6 % slower.  Off: a run-time choice (a kernel argument) costs the
// headline kernel, at its register limit, a scratch spill per round.
#ifndef SEM_XCD_SWIZZLE
#define SEM_XCD_SWIZZLE 0
#endif
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nwg) {
#if SEM_XCD_SWIZZLE
  constexpr int64_t NX = 8;
  const int64_t q = nwg / NX, r = nwg % NX, x = b % NX, k = b / NX;
  return x * q + (x < r ? x : r) + k;
#else
  (void)nwg;
  return b;
#endif
}

// ---------------------------------------------------------------------------
// Poisson stiffness action: one workgroup per chain, chains [c0, c1).
// ---------------------------------------------------------------------------
// minimum waves per SIMD requested from the register allocator.  p = 8
// nodal: 4 (128 VGPRs, no spill; the unpadded tiles fit 4 workgroups per CU)
// measured 0.709 vs 0.731 ms at 3 waves (profiles/r01/occupancy).
// p = 14 stored, seam plan: a 5-wave request (the allocator lands at 3
// waves with a different schedule) measured 0.128-0.129 against 0.135 ms
// per action at 227^2 (natural 4 waves) and 0.132 (3); the same request at
// p = 10 / 12 is 13 % / 40 % slower (profiles/r03/knobs/min_waves/), and it
// would push the colour-launch and fused-dot forms of p = 14 to 2 waves
// (247 / 171 VGPRs), so it applies to the seam form only
// p = 4 nodal colour launches (the instantiation AUTO runs on the cfg4
// mesh): a 6-wave request (98 -> 80 VGPRs, 4 -> 6 waves) measured 0.103-0.105
// against 0.116-0.119 ms per action (call AC, two runs alternating,
// profiles/r03/knobs/min_waves_low/); requests at p = 2 / 6 leave their
// AUTO instantiations' code unchanged, and cfg2 (p = 8 seams) keeps 4.
// Stored-factor seam kernels at n = 12 / 13 / 15 / 17 (with the transposed
// D copy, SEM_DEO_TRANSPOSED, the static register tables: n = 12 natural 126
// VGPRs + 108 SGPRs spilled to lanes, 4-wave request 106 and none; n = 15
// natural 118 / 4 waves, the old 5-wave request 171 / 2 waves; n = 17
// natural 161 + 42 spilled, 3-wave request 136 and none).  Measured on one
// MI355X, kernel median ms per action, two alternating runs each
// (profiles/r04/high_order/): p = 16 198^2 before 0.133 / 0.137, transposed
// copy + 3-wave request 0.137 / 0.140, transposed + natural 0.131 / 0.131;
// p = 14 227^2 0.131 / 0.131 -> 0.129 / 0.129 (natural; the old 5-wave
// request would now give 2 waves); p = 12 263^2 0.128 / 0.124 -> 0.123 /
// 0.124; p = 10 316^2 0.121 / 0.120 -> 0.120 / 0.116.  SEM_MW_S<n>
// overrides the request per order (A/B builds); 0 = the default below.
#ifndef SEM_MW_S12
#define SEM_MW_S12 0
#endif
#ifndef SEM_MW_S13
#define SEM_MW_S13 0
#endif
#ifndef SEM_MW_S15
#define SEM_MW_S15 0
#endif
#ifndef SEM_MW_S17
#define SEM_MW_S17 0
#endif
constexpr int stored_seam_mw(int n) {
  return n == 12 ? (SEM_MW_S12 ? SEM_MW_S12 : (SEM_DEO_TRANSPOSED ? 4 : 1))
       : n == 13 ? (SEM_MW_S13 ? SEM_MW_S13 : 1)
       : n == 15 ? (SEM_MW_S15 ? SEM_MW_S15 : (SEM_DEO_TRANSPOSED ? 1 : 5))
       : n == 17 ? (SEM_MW_S17 ? SEM_MW_S17 : 1)
                 : 1;
}
// the stored seam kernels with D as constants (CD): p = 12 (n = 13) with a
// 5-wave request (96 VGPRs, 16 B of scratch) measured 0.109-0.110 against
// 0.123-0.124 ms per action (natural 4 waves; profiles/r04/const_d/l_*);
// the same request at n = 11 0.117 against 0.108, at n = 15 no change;
// p = 9 (n = 10) with constants and 5 waves 0.1123-0.1125 against
// 0.1141 for the argument form (call N).  SEM_MW_CD_N / _W override one
// order (A/B builds).
#ifndef SEM_MW_CD_N
#define SEM_MW_CD_N 0
#endif
#ifndef SEM_MW_CD_W
#define SEM_MW_CD_W 0
#endif
constexpr int cd_seam_mw(int n) {
  return n == SEM_MW_CD_N ? SEM_MW_CD_W : (n == 13 || n == 10) ? 5 : stored_seam_mw(n);
}
template <int N, bool NODAL, bool SEAM = false, bool DOT = false, bool CD = false>
struct PoissonMinWaves {
  static constexpr int value = SEM_POISSON_MIN_WAVES > 0             ? SEM_POISSON_MIN_WAVES
                               : (CD && !NODAL && SEAM && !DOT)      ? cd_seam_mw(N)
                               : (NODAL && N == 9)                   ? 4
                               : (!NODAL && SEAM && !DOT)            ? stored_seam_mw(N)
                               : (NODAL && N == 5 && !SEAM && !DOT)  ? 6
                                                                     : 1;
};

// RawLaunder: which column-kernel instantiations launder their map entries
// and the wide-group lane offset (chain_emit, load_map).  Static register
// tables (-Rpass-analysis, ScratchSize / VGPRs / waves): the headline
// k_poisson_apply<9, NODAL, M16, SEAM> 12 B of scratch with a store and a
// reload every round -> no scratch access in the round loop (one spill
// before it, one reload in the rare wide-group branch); the n = 9 nodal
// colour-launch form 12 B -> 0; n = 3 / 5 nodal 65 / 80 -> 62 / 72 VGPRs
// (7 -> 8 / 6 -> 7 waves); n = 13 / 17 stored seams 106 / 161 -> 102 / 158.
// Left out: the fused-dot forms (n = 9: 20 -> 36 B of scratch) and n = 11
// (90 -> 105 VGPRs, 5 -> 4 waves).
#ifndef SEM_RAW_LAUNDER
#define SEM_RAW_LAUNDER 1
#endif
template <int N, bool DOT>
struct RawLaunder {
  static constexpr bool value = SEM_RAW_LAUNDER && !DOT && N != 11;
};

struct SeamPlan {
  const uint8_t* __restrict__ colour;  // [chain]
  double* buf;                         // [colour][node]
  int64_t n_node;
  double* dot = nullptr;  // DOT kernels: one partial of u.y per workgroup
  int round_sync = 1;     // a chain writes some node in two rounds: order the rounds
  const double* w = nullptr;  // device copy of the weights (SEM_W_SCALAR_LOAD)
};

// sum of one value per thread over the workgroup, in a fixed order (wave
// reductions, then the waves in order), returned by thread 0
template <int NW>
__device__ __forceinline__ double block_sum_fixed(double v, double* sh) {
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) v += __shfl_down(v, o, WAVE);
  if (threadIdx.x % WAVE == 0) sh[threadIdx.x / WAVE] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
#pragma unroll
    for (int w = 0; w < NW; ++w) s += sh[w];
  return s;
}

template <int N, bool NODAL, bool M16, bool SEAM = false, bool DOT = false, bool CD = false,
          bool PAT = false>
__global__ void __launch_bounds__(ChainWaves<N>::block, (PoissonMinWaves<N, NODAL, SEAM, DOT, CD>::value))
    k_poisson_apply(const MapRef mref, const double* __restrict__ GP,
                    const double2* __restrict__ XG, const double* __restrict__ u,
                    double* __restrict__ y, int64_t c0, int64_t c1, int rounds, int accumulate,
                    const DEO<N> Darg, const WVec<N> w, const SeamPlan sp) {
  const auto D = deo_view<N, CD>(Darg);
  using T = Tile<N, NODAL ? SEM_TILE_PAD_NODAL : stored_pad(N)>;
  constexpr int NT = NODAL ? 2 : 1;  // tiles per element slot
  constexpr int CW = ChainWaves<N>::value;
  constexpr bool WL = NODAL ? NodalTile<N>::wl : StoredTile<N>::wl;
  constexpr int PLANE = WL ? CW * WLTile<N>::WS : T::TILE_SLOTS * T::ES;  // doubles per tile plane
  __shared__ __attribute__((aligned(16))) double lds[PLANE * NT];
  __shared__ double carry[CARRY_BUFS][CW][1][N];
  const int64_t chain = c0 + xcd_block(blockIdx.x, gridDim.x);
  if (chain >= c1) {  // uniform over the workgroup
    if constexpr (DOT)
      if (threadIdx.x == 0) sp.dot[blockIdx.x] = 0.0;
    return;
  }
  double dotv = 0.0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);  // provably uniform
  const int lane = threadIdx.x % WAVE;
  const int k = lane / N;
  const int j = lane - k * N;
  const bool in_wave = lane < T::LW;
  // tile planes: all of tile A, then all of tile B (interleaving A/B per
  // slot doubles the stride and makes the column accesses 2-way bank
  // conflicts)
  double* L = lds + (WL ? WLTile<N>::base(wave, k) : T::slot(wave, k, in_wave) * T::ES);
  double* LB = L + (NT - 1) * PLANE;
  const double wj = pick<N>(w, j);
  double rowc[1] = {0.0};
  for (int rd = 0; rd < rounds; ++rd) {
    const int64_t g = (chain * rounds + rd) * CW + wave;
    uint32_t raw[N];
    double v[1][N], prev[N];
    constexpr bool TOUCH = SEM_MAP_TOUCH && M16 && !DOT;
    MapTouch<N> touch;
    if constexpr (TOUCH)
      if (rd + 1 < rounds) touch.issue(mref, g + CW, lane);
    using Pre = typename std::conditional<SEAM, NoPrefetch, NoWait>::type;
    const Pre pre{};
    constexpr bool PRE = RmwPrefetch<N>::value > 0 && Pre::prefetch;
    constexpr bool LD = RawLaunder<N, DOT>::value;
    if constexpr (NODAL)
      poisson_group_nodal<N, M16, Pre, LD, PAT>(mref, XG, u, g, lane, j, in_wave, L, LB, D, w, wj, raw,
                                           v[0], y, accumulate, prev, pre, sp.w);
    else
      poisson_group_stored<N, M16, Pre, LD, PAT>(mref, GP, u, g, lane, j, in_wave, L, D, raw, v[0], y,
                                            accumulate, prev, pre);
    SeamOut so;
    if constexpr (SEAM) so.base = sp.buf + sp.colour[chain] * sp.n_node;
    chain_emit<N, 1, PRE, CW, SEAM, DOT, LD, CD>(y, raw, v, lane, wave, rd, in_wave, carry, rowc,
                                         accumulate, sp.round_sync, prev, so, u, &dotv);
    if constexpr (TOUCH)
      if (rd + 1 < rounds) touch.done();
  }
  if constexpr (DOT) {
    __shared__ double sh[CW];
    const double t = block_sum_fixed<CW>(dotv, sh);
    if (threadIdx.x == 0) sp.dot[blockIdx.x] = t;
  }
}

// second launch of the seam plan: y[gid] (+)= the colour slots, in colour
// order (the order of the colour launches' read-modify-writes: the same
// rounding).  mask bits 0-7: colours that wrote the node; bit 8: y already
// holds a value (SEM_NODE_PRIOR)
// NS colours: the slot loads of a node are issued together (predicated
// buffer loads: an unused slot reads past the range, 0 and no traffic).
// nodes per thread per pass: 2 measured slower at p = 8 (41.5-41.8 against
// 36.7-39.3 us per seam sum) and faster at p = 16 (10.0-10.2 against
// 11.2-11.6), 4 no better (profiles/r03/knobs/seam_ilp.txt)
#ifndef SEAM_ILP
#define SEAM_ILP 1
#endif
// per context (seam_ilp_of): 2 at n = 17, where it measured faster per
// action with the constant-D kernel: 0.1270-0.1275 against 0.1277-0.1288 ms
// per step, three runs alternating (profiles/r04/knobs_high/x_*, u_*)
#ifndef SEAM_ILP_17
#define SEAM_ILP_17 2
#endif
template <int NS, bool DOT = false, int ILP = SEAM_ILP>
__global__ void __launch_bounds__(BLOCK)
    k_seam_sum(double* __restrict__ y, const uint32_t* __restrict__ gid,
               const uint16_t* __restrict__ mask, int64_t n, const double* __restrict__ buf,
               int64_t n_node, int accumulate, const double* __restrict__ du = nullptr,
               double* __restrict__ dot = nullptr);

// two DOFs per node (axisymmetric block): slots are double2, buf[colour][node]
template <int NS>
__global__ void k_seam_sum2(double* __restrict__ y, const uint32_t* __restrict__ gid,
                            const uint16_t* __restrict__ mask, int64_t n,
                            const double* __restrict__ buf, int64_t n_node, int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = gid[i];
    const uint32_t m = mask[i];
    const bool prior = accumulate || (m & 0x100u);
    double2 s = prior ? reinterpret_cast<const double2*>(y)[g] : make_double2(0.0, 0.0);
    bool first = !prior;
#pragma unroll
    for (int c = 0; c < NS; ++c)
      if (m & (1u << c)) {
        const double2 b = reinterpret_cast<const double2*>(buf + 2 * c * n_node)[g];
        s = first ? b : make_double2(s.x + b.x, s.y + b.y);
        first = false;
      }
    reinterpret_cast<double2*>(y)[g] = s;
  }
}

template <int NS, bool DOT, int ILP>
__global__ void __launch_bounds__(BLOCK)
    k_seam_sum(double* __restrict__ y, const uint32_t* __restrict__ gid,
               const uint16_t* __restrict__ mask, int64_t n, const double* __restrict__ buf,
               int64_t n_node, int accumulate, const double* __restrict__ du,
               double* __restrict__ dot) {
  // ILP nodes per thread per pass (a block covers ILP * BLOCK
  // consecutive seam nodes): their index, slot and y loads are in flight
  // together instead of one dependent chain per node
  double dotv = 0.0;
  // one buffer resource per colour plane (each < 2^31 bytes: n_node < 2^28)
  __amdgpu_buffer_rsrc_t rb[NS];
#pragma unroll
  for (int c = 0; c < NS; ++c)
    rb[c] = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(buf + c * n_node), 0, 0x80000000,
                                              0x00020000);
  for (int64_t b0 = (int64_t)blockIdx.x * (ILP * BLOCK); b0 < n;
       b0 += (int64_t)gridDim.x * (ILP * BLOCK)) {
    uint32_t g[ILP], m[ILP];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const int64_t i = b0 + q * BLOCK + threadIdx.x;
      const bool in = i < n;
      g[q] = in ? gid[i] : 0u;
      m[q] = in ? (uint32_t)mask[i] : 0u;
    }
    double y0[ILP], b[ILP][NS];
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      const bool prior = m[q] && (accumulate || (m[q] & 0x100u));
      y0[q] = prior ? y[g[q]] : 0.0;
#pragma unroll
      for (int c = 0; c < NS; ++c) {
        const uint32_t off = (m[q] & (1u << c)) ? g[q] * 8u : 0x80000000u;
        b[q][c] =
            __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rb[c], off, 0, CPOL_NT));
      }
    }
#pragma unroll
    for (int q = 0; q < ILP; ++q) {
      if (!m[q]) continue;  // past the end
      const bool prior = accumulate || (m[q] & 0x100u);
      double s = y0[q];
      bool first = !prior;
#pragma unroll
      for (int c = 0; c < NS; ++c)
        if (m[q] & (1u << c)) {
          s = first ? b[q][c] : s + b[q][c];
          first = false;
        }
      y[g[q]] = s;
      if constexpr (DOT) dotv = fma(du[g[q]], s, dotv);
    }
  }
  if constexpr (DOT) {
    __shared__ double sh[BLOCK / WAVE];
    const double t = block_sum_fixed<BLOCK / WAVE>(dotv, sh);
    if (threadIdx.x == 0) dot[blockIdx.x] = t;
  }
}

// The decomposition's finish fused with the interior's seam sum
// (sem::ctx_seam_finish, sem_dd.hip).  t < n: seam node g, s = its slots in
// colour order as k_seam_sum, plus -- when the interface also touches g --
// v = y_c + the neighbours' values in peer order (the order of the unfused
// seam sum, then y = y + v); then the interface DOFs off the seams and the
// deferred zero list as k_dd_finish.  Bitwise equal to the two launches.
template <int NS>
__global__ void __launch_bounds__(BLOCK)
    k_seam_dd_finish(double* __restrict__ y, const uint32_t* __restrict__ gid,
                     const uint16_t* __restrict__ mask, int64_t n, const double* __restrict__ buf,
                     int64_t n_node, const sem::DDFinish f) {
  auto iface_value = [&](int64_t j, uint32_t i) {
    double v = f.yc[f.yc_local ? i : j];
    for (int32_t k = f.rp[j]; k < f.rp[j + 1]; ++k) v += f.recv[f.rpos[k]];
    return v;
  };
  // one buffer resource per colour plane, slot loads issued together
  // (predicated: an unused slot reads past the range, 0 and no traffic), as
  // in k_seam_sum
  __amdgpu_buffer_rsrc_t rb[NS];
#pragma unroll
  for (int c = 0; c < NS; ++c)
    rb[c] = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(buf + c * n_node), 0, 0x80000000,
                                              0x00020000);
  const int64_t ns = f.sel ? f.n_sel : n;
  const int64_t nr = f.skip_rest ? 0 : f.n_rest;
  const int64_t nzl = f.skip_zero ? 0 : f.nz;
  const int64_t tot = ns + nr + nzl;
  for (int64_t ti = blockIdx.x * (int64_t)BLOCK + threadIdx.x; ti < tot;
       ti += (int64_t)gridDim.x * BLOCK) {
    if (ti < ns) {
      const int64_t t = f.sel ? (int64_t)f.sel[ti] : ti;
      const uint32_t g = gid[t];
      const uint32_t m = mask[t];
      const bool prior = (m & 0x100u) != 0;
      double b[NS];
#pragma unroll
      for (int c = 0; c < NS; ++c) {
        const uint32_t off = (m & (1u << c)) ? g * 8u : 0x80000000u;
        b[c] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rb[c], off, 0, CPOL_NT));
      }
      double s = prior ? y[g] : 0.0;
      bool first = !prior;
#pragma unroll
      for (int c = 0; c < NS; ++c)
        if (m & (1u << c)) {
          s = first ? b[c] : s + b[c];
          first = false;
        }
      const int32_t j = f.seam_cj[t];
      if (j >= 0) s = s + iface_value(j, g);
      y[g] = s;
    } else if (ti < ns + nr) {
      const uint32_t j = f.rest[ti - ns];
      const uint32_t e = f.fidx[j];
      const uint32_t i = e & 0x7fffffffu;
      const double v = iface_value(j, i);
      y[i] = ((e >> 31) ? 0.0 : y[i]) + v;
    } else {
      y[f.fzero[ti - ns - nr]] = 0.0;
    }
  }
}

// The interface context's seam sum fused with the pack of the send buffer
// (sem::ctx_seam_pack, sem_dd.hip dd_side): t < n: seam node g of the
// interface plan, y_c[g] = its colour slots in colour order (k_seam_sum,
// overwrite mode); then send[k] = y_c[sidx[k]] for every exchanged DOF, the
// value of a seam node formed again from its slots (sj[k] = its seam index)
// rather than read back, so no thread waits for another.  Bitwise equal to
// the seam-sum launch followed by the gather; seam nodes with a prior value
// (SEM_NODE_PRIOR) are not fused (the caller checks).
template <int NS>
__global__ void __launch_bounds__(BLOCK)
    k_seam_pack(double* __restrict__ y, const uint32_t* __restrict__ gid,
                const uint16_t* __restrict__ mask, int64_t n, const double* __restrict__ buf,
                int64_t n_node, double* __restrict__ send, const uint32_t* __restrict__ sidx,
                const int32_t* __restrict__ sj, int64_t ne) {
  __amdgpu_buffer_rsrc_t rb[NS];
#pragma unroll
  for (int c = 0; c < NS; ++c)
    rb[c] = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(buf + c * n_node), 0, 0x80000000,
                                              0x00020000);
  auto seam_value = [&](int64_t t, uint32_t g) {
    const uint32_t m = mask[t];
    double b[NS];
#pragma unroll
    for (int c = 0; c < NS; ++c) {
      const uint32_t off = (m & (1u << c)) ? g * 8u : 0x80000000u;
      b[c] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rb[c], off, 0, CPOL_NT));
    }
    double s = 0.0;
    bool first = true;
#pragma unroll
    for (int c = 0; c < NS; ++c)
      if (m & (1u << c)) {
        s = first ? b[c] : s + b[c];
        first = false;
      }
    return s;
  };
  const int64_t tot = n + ne;
  for (int64_t t = blockIdx.x * (int64_t)BLOCK + threadIdx.x; t < tot;
       t += (int64_t)gridDim.x * BLOCK) {
    if (t < n) {
      const uint32_t g = gid[t];
      y[g] = seam_value(t, g);
    } else {
      const int64_t k = t - n;
      const int32_t j = sj[k];
      send[k] = j >= 0 ? seam_value(j, gid[j]) : y[sidx[k]];
    }
  }
}

// fixed-order sum of the DOT partials of an action: na chain partials, then
// nb seam-sum partials -> *out.  One workgroup of DOT_FIN_THREADS: thread t
// sums entries t, t + T, ... in order (17.7K partials at 1024^2, 17 each),
// then a fixed-order workgroup sum.  (256 threads, 69 entries each: 22.9 us
// per PCG iteration, profiles/r05/pcg/.)
constexpr int DOT_FIN_THREADS = 1024;
[[maybe_unused]] static __global__ void __launch_bounds__(DOT_FIN_THREADS)
    k_dot_finish(const double* __restrict__ a, int64_t na, const double* __restrict__ b,
                 int64_t nb, double* __restrict__ out) {
  double v = 0.0;
  for (int64_t i = threadIdx.x; i < na; i += DOT_FIN_THREADS) v += a[i];
  for (int64_t i = threadIdx.x; i < nb; i += DOT_FIN_THREADS) v += b[i];
  __shared__ double sh[DOT_FIN_THREADS / WAVE];
  const double t = block_sum_fixed<DOT_FIN_THREADS / WAVE>(v, sh);
  if (threadIdx.x == 0) *out = t;
}


// ---------------------------------------------------------------------------
// Axisymmetric Stokes block (Re = 0), dpn = 2 interleaved (psi, omega):
//   y[2k]   = Lve.omega          = stiff_rho(omega) + (W/rho) omega
//   y[2k+1] = E2e.psi - Me.omega = stiff_rho(psi) + 2W(iJ00 d0 + iJ10 d1)psi - rho^2 W omega
// (examples/squirmer-axisymmetric.py:193-227, 253-254, 278-295)
// factors: 0 G00rho 1 G01rho 2 G11rho 3 b0=2W iJ00 4 b1=2W iJ10 5 c=W/rho 6 m=rho^2 W
// Navier-Stokes (MODE 1 residual, MODE 2 Jacobian-vector product) adds
// 7 (W/rho) iJ01, 8 (W/rho) iJ11 and the advection term Ae (squirmer:229-250)
// at test node (m, j) of the omega row:
//   Re [ w_m w_j (d0 psi d1 w - d1 psi d0 w) + w (f7 d0 psi + f8 d1 psi) ]
// MODE 1 can record its linearisation a0..a4 per element node (LIN):
//   J.delta|omega row += a0 d0 dpsi + a1 d1 dpsi + a2 d0 dw + a3 d1 dw + a4 dw
// ---------------------------------------------------------------------------
struct AxiNS {
  double re = 0.0;
  double* lin = nullptr;  // MODE 1: write, MODE 2: read; [slot][5][r][lane]
};

template <int N, int MODE>
__device__ __forceinline__ void axisym_group(const uint32_t* __restrict__ mapP,
                                             const double* __restrict__ GP,
                                             const double* __restrict__ u, int64_t g, int lane,
                                             int j, bool in_wave, double* LP, double* LO,
                                             const DEO<N>& D, const WVec<N>& w, double wj,
                                             const AxiNS& ns, uint32_t (&raw)[N],
                                             double (&vo)[N], double (&vp)[N]) {
  using T = Tile<N>;
  constexpr int LW = T::LW;
  constexpr int RS = T::RS;
  constexpr int NF = MODE ? 9 : 7;
  const uint32_t* mp = mapP + g * (int64_t)(N * LW) + lane;
  const double* gp = GP + g * (int64_t)(NF * N * LW) + lane;
  double* lin = MODE ? ns.lin + g * (int64_t)(5 * N * LW) + lane : nullptr;
  const double2* u2 = reinterpret_cast<const double2*>(u);
  double ps[N], om[N];
#pragma unroll
  for (int r = 0; r < N; ++r) raw[r] = in_wave ? mp[r * LW] : (W_SKIP << CODE_SHIFT);
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const double2 val = u2[raw[r] & GID_MASK];
    ps[r] = val.x;
    om[r] = val.y;
  }
  double d0p[N], d0o[N];
  deo_apply<N>(D, ps, d0p);
  deo_apply<N>(D, om, d0o);
#pragma unroll
  for (int r = 0; r < N; ++r) {
    LP[r * RS + j] = ps[r];
    LO[r * RS + j] = om[r];
  }
  wave_sync();
  {
    double tp[N], to[N];
    double rp[RS], ro[RS], xp[N], xo[N];
    load_row<N, RS>(LP, j, rp);
    load_row<N, RS>(LO, j, ro);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      xp[q] = rp[q];
      xo[q] = ro[q];
    }
    deo_apply<N>(D, xp, tp);
    deo_apply<N>(D, xo, to);
    wave_sync();
    store_row<N, RS>(LP, j, tp);
    store_row<N, RS>(LO, j, to);
  }
  wave_sync();
  double w1p[N], w1o[N];
  {
    double w0p[N], w0o[N];
#pragma unroll
    for (int m = 0; m < N; ++m) {
      const double d1p = LP[m * RS + j];
      const double d1o = LO[m * RS + j];
      const double g00 = gp[(0 * N + m) * LW];
      const double g01 = gp[(1 * N + m) * LW];
      const double g11 = gp[(2 * N + m) * LW];
      const double b0 = gp[(3 * N + m) * LW];
      const double b1 = gp[(4 * N + m) * LW];
      const double c = gp[(5 * N + m) * LW];
      const double mm = gp[(6 * N + m) * LW];
      w0p[m] = fma(g00, d0p[m], g01 * d1p);
      w1p[m] = fma(g01, d0p[m], g11 * d1p);
      w0o[m] = fma(g00, d0o[m], g01 * d1o);
      w1o[m] = fma(g01, d0o[m], g11 * d1o);
      // pointwise terms at test node (m, j): psi row 2W gx(psi) - rho^2 W omega,
      // omega row (W/rho) omega (+ the advection term for Navier-Stokes)
      double adv = 0.0;
      if constexpr (MODE == 1) {
        const double f7 = gp[(7 * N + m) * LW], f8 = gp[(8 * N + m) * LW];
        const double rw = ns.re * (w.v[m] * wj);
        const double dz = fma(f7, d0p[m], f8 * d1p);  // (W/rho) dpsi/dz
        adv = fma(rw, fma(d0p[m], d1o, -d1p * d0o[m]), ns.re * om[m] * dz);
        if (lin && in_wave) {
          lin[(0 * N + m) * LW] = fma(rw, d1o, ns.re * f7 * om[m]);
          lin[(1 * N + m) * LW] = fma(-rw, d0o[m], ns.re * f8 * om[m]);
          lin[(2 * N + m) * LW] = -rw * d1p;
          lin[(3 * N + m) * LW] = rw * d0p[m];
          lin[(4 * N + m) * LW] = ns.re * dz;
        }
      } else if constexpr (MODE == 2) {
        adv = fma(lin[(0 * N + m) * LW], d0p[m],
                  fma(lin[(1 * N + m) * LW], d1p,
                      fma(lin[(2 * N + m) * LW], d0o[m],
                          fma(lin[(3 * N + m) * LW], d1o, lin[(4 * N + m) * LW] * om[m]))));
      }
      d0p[m] = fma(b0, d0p[m], fma(b1, d1p, -mm * om[m]));
      d0o[m] = fma(c, om[m], adv);
    }
    deo_apply_t<N>(D, w0p, vp);
    deo_apply_t<N>(D, w0o, vo);
#pragma unroll
    for (int p = 0; p < N; ++p) {
      vp[p] += d0p[p];
      vo[p] += d0o[p];
    }
  }
  wave_sync();
#pragma unroll
  for (int m = 0; m < N; ++m) {
    LP[m * RS + j] = w1p[m];
    LO[m * RS + j] = w1o[m];
  }
  wave_sync();
  {
    double tp[N], to[N];
    double rp[RS], ro[RS], xp[N], xo[N];
    load_row<N, RS>(LP, j, rp);
    load_row<N, RS>(LO, j, ro);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      xp[q] = rp[q];
      xo[q] = ro[q];
    }
    deo_apply_t<N>(D, xp, tp);
    deo_apply_t<N>(D, xo, to);
    wave_sync();
    store_row<N, RS>(LP, j, tp);
    store_row<N, RS>(LO, j, to);
  }
  wave_sync();
#pragma unroll
  for (int p = 0; p < N; ++p) {
    vo[p] += LO[p * RS + j];
    vp[p] += LP[p * RS + j];
  }
  wave_sync();
}

// ---------------------------------------------------------------------------
// Axisymmetric Stokes block with NODAL geometry: the seven factors of the
// lane's column are re-derived per node from x_phys per global node, as in
// the Poisson NODAL group (J along the column in registers, along the row
// through the tiles, coordinates relative to the line's first node), with
// rho = x (squirmer-axisymmetric.py:193-227).  With ww = w_m w_j:
//   G..rho = rho (ww / det) (the Poisson combinations of J),
//   b0 = 2 W iJ00 = 2 ww J11,   b1 = 2 W iJ10 = -2 ww J10,
//   c = W / rho,   m = rho^2 W,   W = ww det.
// 16 B of x_phys per node replace 56 B of factors per element node.
// ---------------------------------------------------------------------------
#ifndef SEM_AXI_MIN_WAVES
#define SEM_AXI_MIN_WAVES 1
#endif
#ifndef SEM_AXI_EARLY_U
#define SEM_AXI_EARLY_U 0
#endif
template <int N, bool M16, bool PAT = false>
__device__ __forceinline__ void axisym_group_nodal(const MapRef& mref,
                                                   const double2* __restrict__ XG,
                                                   const double* __restrict__ u, int64_t g,
                                                   int lane, int j, bool in_wave, double* LP,
                                                   double* LO, const DEO<N>& D, const WVec<N>& w,
                                                   double wj, uint32_t (&raw)[N], double (&vo)[N],
                                                   double (&vp)[N]) {
  constexpr int RS = Tile<N>::RS;
  load_map<N, M16, false, PAT>(mref, g, lane, in_wave, raw);
  double2 xc[N];
  gather_x<N>(XG, raw, j, xc);
  const double2* u2 = reinterpret_cast<const double2*>(u);
  double ps[N], om[N];
#if SEM_AXI_EARLY_U
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const double2 val = u2[raw[r] & GID_MASK];
    ps[r] = val.x;
    om[r] = val.y;
  }
#endif
  // Jacobian: jr = d(x, y)/dr along the column, js = d(x, y)/ds along the row
  double jr0[N], jr1[N], js0[N], js1[N], rho[N];
  {
    double ta[N], tb[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
      ta[r] = xc[r].x - xc[0].x;
      tb[r] = xc[r].y - xc[0].y;
      rho[r] = xc[r].x;
    }
    deo_apply<N>(D, ta, jr0);
    deo_apply<N>(D, tb, jr1);
  }
#pragma unroll
  for (int r = 0; r < N; ++r) {
    LP[r * RS + j] = xc[r].x;
    LO[r * RS + j] = xc[r].y;
  }
  wave_sync();
  {
    double xa[RS], xb[RS], ra[N], rb[N], ta[N], tb[N];
    load_row<N, RS>(LP, j, xa);
    load_row<N, RS>(LO, j, xb);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      ra[q] = xa[q] - xa[0];
      rb[q] = xb[q] - xb[0];
    }
    deo_apply<N>(D, ra, ta);
    deo_apply<N>(D, rb, tb);
    wave_sync();
    store_row<N, RS>(LP, j, ta);
    store_row<N, RS>(LO, j, tb);
  }
  wave_sync();
  // own column slots: read js, then the same lane rewrites them with psi/omega
#pragma unroll
  for (int m = 0; m < N; ++m) {
    js0[m] = LP[m * RS + j];
    js1[m] = LO[m * RS + j];
  }
#if !SEM_AXI_EARLY_U
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const double2 val = u2[raw[r] & GID_MASK];
    ps[r] = val.x;
    om[r] = val.y;
  }
#endif
  double d0p[N], d0o[N];
  deo_apply<N>(D, ps, d0p);
  deo_apply<N>(D, om, d0o);
#pragma unroll
  for (int r = 0; r < N; ++r) {
    LP[r * RS + j] = ps[r];
    LO[r * RS + j] = om[r];
  }
  wave_sync();
  {
    double rp[RS], ro[RS], xp[N], xo[N], tp[N], to[N];
    load_row<N, RS>(LP, j, rp);
    load_row<N, RS>(LO, j, ro);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      xp[q] = rp[q];
      xo[q] = ro[q];
    }
    deo_apply<N>(D, xp, tp);
    deo_apply<N>(D, xo, to);
    wave_sync();
    store_row<N, RS>(LP, j, tp);
    store_row<N, RS>(LO, j, to);
  }
  wave_sync();
#pragma unroll
  for (int m = 0; m < N; ++m) {
    const double d1p = LP[m * RS + j];
    const double d1o = LO[m * RS + j];
    const double det = jr0[m] * js1[m] - js0[m] * jr1[m];
    const double wm = w.v[m];
    const double rs = rho[m] * (wm * (wj * fast_rcp(det)));
    const double g00 = rs * fma(js1[m], js1[m], js0[m] * js0[m]);
    const double g01 = -rs * fma(js1[m], jr1[m], js0[m] * jr0[m]);
    const double g11 = rs * fma(jr1[m], jr1[m], jr0[m] * jr0[m]);
    const double W = wm * (wj * det);
    const double b0 = 2.0 * wm * (wj * js1[m]);
    const double b1 = -2.0 * wm * (wj * jr1[m]);
    const double c = W * fast_rcp(rho[m]);
    const double mm = rho[m] * rho[m] * W;
    // w1 -> own slot (read above); w0 and the pointwise terms stay in registers
    LP[m * RS + j] = fma(g01, d0p[m], g11 * d1p);
    LO[m * RS + j] = fma(g01, d0o[m], g11 * d1o);
    vp[m] = fma(b0, d0p[m], fma(b1, d1p, -mm * om[m]));
    vo[m] = c * om[m];
    d0p[m] = fma(g00, d0p[m], g01 * d1p);
    d0o[m] = fma(g00, d0o[m], g01 * d1o);
  }
  {
    double tp[N], to[N];
    deo_apply_t<N>(D, d0p, tp);
    deo_apply_t<N>(D, d0o, to);
#pragma unroll
    for (int p = 0; p < N; ++p) {
      vp[p] += tp[p];
      vo[p] += to[p];
    }
  }
  wave_sync();
  {
    double rp[RS], ro[RS], xp[N], xo[N], tp[N], to[N];
    load_row<N, RS>(LP, j, rp);
    load_row<N, RS>(LO, j, ro);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      xp[q] = rp[q];
      xo[q] = ro[q];
    }
    deo_apply_t<N>(D, xp, tp);
    deo_apply_t<N>(D, xo, to);
    wave_sync();
    store_row<N, RS>(LP, j, tp);
    store_row<N, RS>(LO, j, to);
  }
  wave_sync();
#pragma unroll
  for (int p = 0; p < N; ++p) {
    vo[p] += LO[p * RS + j];
    vp[p] += LP[p * RS + j];
  }
  wave_sync();
}

// The same group, fields first (round 3): psi / omega are gathered and
// differentiated before the geometry, d1 of both fields waits in the two
// field tiles while the geometry runs through a third tile plane (x, then
// y), so the Jacobian arrays never coexist with the row-pass temporaries of
// the fields -- the live set drops from 256 VGPRs (one or two waves per SIMD)
// to the three-wave range.  Same arithmetic, same order per node as
// axisym_group_nodal.
#ifndef SEM_AXI_FIELDS_FIRST
#define SEM_AXI_FIELDS_FIRST 1
#endif
template <int N, bool M16, bool PAT = false>
__device__ __forceinline__ void axisym_group_nodal3(const MapRef& mref,
                                                    const double2* __restrict__ XG,
                                                    const double* __restrict__ u, int64_t g,
                                                    int lane, int j, bool in_wave, double* LP,
                                                    double* LO, double* LG, const DEO<N>& D,
                                                    const WVec<N>& w, double wj,
                                                    uint32_t (&raw)[N], double (&vo)[N],
                                                    double (&vp)[N]) {
  constexpr int RS = Tile<N>::RS;
  constexpr bool SP = SEM_LDS_SPLIT_AXI;
  load_map<N, M16, false, PAT>(mref, g, lane, in_wave, raw);
  const double2* u2 = reinterpret_cast<const double2*>(u);
  double om[N], d0p[N], d0o[N];
  {
    double ps[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
      const double2 val = u2[raw[r] & GID_MASK];
      ps[r] = val.x;
      om[r] = val.y;
    }
    deo_apply<N>(D, ps, d0p);
    deo_apply<N>(D, om, d0o);
#pragma unroll
    for (int r = 0; r < N; ++r) {
      LP[r * RS + j] = ps[r];
      LO[r * RS + j] = om[r];
    }
  }
  wave_sync();
  row_pass<N, RS, false, false>(LP, j, D);  // d1 psi
  row_pass<N, RS, false, false>(LO, j, D);  // d1 omega
  // geometry: J along the column in registers, along the row through LG
  double jr0[N], jr1[N], js0[N], js1[N], rho[N];
  {
    double2 xc[N];
    gather_x<N>(XG, raw, j, xc);
    double ta[N], tb[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
      ta[r] = xc[r].x - xc[0].x;
      tb[r] = xc[r].y - xc[0].y;
      rho[r] = xc[r].x;
      LG[r * RS + j] = xc[r].x;
    }
    deo_apply<N>(D, ta, jr0);
    deo_apply<N>(D, tb, jr1);
    wave_sync();
    row_pass<N, RS, false, true>(LG, j, D);
#pragma unroll
    for (int m = 0; m < N; ++m) js0[m] = lds_ld<SP>(LG + m * RS + j);
    wave_sync();
#pragma unroll
    for (int r = 0; r < N; ++r) LG[r * RS + j] = xc[r].y;
  }
  wave_sync();
  row_pass<N, RS, false, true>(LG, j, D);
#pragma unroll
  for (int m = 0; m < N; ++m) js1[m] = lds_ld<SP>(LG + m * RS + j);
  // pointwise (squirmer-axisymmetric.py:193-227), as axisym_group_nodal
#pragma unroll
  for (int m = 0; m < N; ++m) {
    const double d1p = lds_ld<SP>(LP + m * RS + j);
    const double d1o = lds_ld<SP>(LO + m * RS + j);
    const double det = jr0[m] * js1[m] - js0[m] * jr1[m];
    const double wm = w.v[m];
    const double rs = rho[m] * (wm * (wj * fast_rcp(det)));
    const double g00 = rs * fma(js1[m], js1[m], js0[m] * js0[m]);
    const double g01 = -rs * fma(js1[m], jr1[m], js0[m] * jr0[m]);
    const double g11 = rs * fma(jr1[m], jr1[m], jr0[m] * jr0[m]);
    const double W = wm * (wj * det);
    const double b0 = 2.0 * wm * (wj * js1[m]);
    const double b1 = -2.0 * wm * (wj * jr1[m]);
    const double c = W * fast_rcp(rho[m]);
    const double mm = rho[m] * rho[m] * W;
    LP[m * RS + j] = fma(g01, d0p[m], g11 * d1p);
    LO[m * RS + j] = fma(g01, d0o[m], g11 * d1o);
    vp[m] = fma(b0, d0p[m], fma(b1, d1p, -mm * om[m]));
    vo[m] = c * om[m];
    d0p[m] = fma(g00, d0p[m], g01 * d1p);
    d0o[m] = fma(g00, d0o[m], g01 * d1o);
  }
  {
    double t[N];
    deo_apply_t<N>(D, d0p, t);
#pragma unroll
    for (int p = 0; p < N; ++p) vp[p] += t[p];
    deo_apply_t<N>(D, d0o, t);
#pragma unroll
    for (int p = 0; p < N; ++p) vo[p] += t[p];
  }
  wave_sync();
  row_pass<N, RS, true, false>(LP, j, D);
  row_pass<N, RS, true, false>(LO, j, D);
#pragma unroll
  for (int p = 0; p < N; ++p) {
    vo[p] += lds_ld<SP>(LO + p * RS + j);
    vp[p] += lds_ld<SP>(LP + p * RS + j);
  }
  wave_sync();
}

// fields first up to n = 8 (three tile planes at three workgroups per CU:
// 151 KB of LDS at n = 7); above, the LDS of a third plane would cost more
// occupancy than the registers gain
template <int N>
struct AxiNodal {
  static constexpr bool fields_first = SEM_AXI_FIELDS_FIRST && N <= 8;
  static constexpr int planes = fields_first ? 3 : 2;
  static constexpr int waves = fields_first ? (SEM_AXI_MIN_WAVES > 1 ? SEM_AXI_MIN_WAVES : 3)
                                            : SEM_AXI_MIN_WAVES;
};

template <int N, bool M16, bool SEAM = false, bool PAT = false>
__global__ void __launch_bounds__(ChainWaves<N>::block, AxiNodal<N>::waves)
    k_axisym_nodal(const MapRef mref, const double2* __restrict__ XG, const double* __restrict__ u,
                   double* __restrict__ y, int64_t c0, int64_t c1, int rounds, int accumulate,
                   const DEO<N> D, const WVec<N> w, const SeamPlan sp) {
  using T = Tile<N>;
  constexpr int NPL = AxiNodal<N>::planes;  // tile planes
  __shared__ __attribute__((aligned(16))) double lds[T::TILE_SLOTS * NPL * T::ES];
  constexpr int CW = ChainWaves<N>::value;
  __shared__ double carry[CARRY_BUFS][CW][2][N];
  const int64_t chain = c0 + blockIdx.x;
  if (chain >= c1) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int lane = threadIdx.x % WAVE;
  const int k = lane / N;
  const int j = lane - k * N;
  const bool in_wave = lane < T::LW;
  const double wj = pick<N>(w, j);
  double* LP = lds + T::slot(wave, k, in_wave) * T::ES;
  double* LO = LP + T::TILE_SLOTS * T::ES;
  double rowc[2] = {0.0, 0.0};
  for (int rd = 0; rd < rounds; ++rd) {
    const int64_t g = (chain * rounds + rd) * CW + wave;
    uint32_t raw[N];
    double v[2][N];  // [0] omega row (y[2k]), [1] psi row (y[2k+1])
    if constexpr (AxiNodal<N>::fields_first)
      axisym_group_nodal3<N, M16, PAT>(mref, XG, u, g, lane, j, in_wave, LP, LO,
                                  LO + T::TILE_SLOTS * T::ES, D, w, wj, raw, v[0], v[1]);
    else
      axisym_group_nodal<N, M16, PAT>(mref, XG, u, g, lane, j, in_wave, LP, LO, D, w, wj, raw, v[0],
                                 v[1]);
    SeamOut so;
    if constexpr (SEAM) so.base = sp.buf + sp.colour[chain] * sp.n_node * 2;
    chain_emit<N, 2, false, CW, SEAM>(y, raw, v, lane, wave, rd, in_wave, carry, rowc, accumulate,
                                      sp.round_sync, nullptr, so);
  }
}

template <int N, int MODE, bool SEAM = false>
__global__ void __launch_bounds__(ChainWaves<N>::block)
    k_axisym_apply(const uint32_t* __restrict__ mapP, const double* __restrict__ GP,
                   const double* __restrict__ u, double* __restrict__ y, int64_t c0, int64_t c1,
                   int rounds, int accumulate, const DEO<N> D, const WVec<N> w, const AxiNS ns,
                   const SeamPlan sp) {
  using T = Tile<N>;
  __shared__ __attribute__((aligned(16))) double lds[T::TILE_SLOTS * 2 * T::ES];
  constexpr int CW = ChainWaves<N>::value;
  __shared__ double carry[CARRY_BUFS][CW][2][N];
  const int64_t chain = c0 + blockIdx.x;
  if (chain >= c1) return;
  const int wave = threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  const int k = lane / N;
  const int j = lane - k * N;
  const bool in_wave = lane < T::LW;
  const double wj = pick<N>(w, j);
  double* LP = lds + T::slot(wave, k, in_wave) * T::ES;  // psi tile plane
  double* LO = LP + T::TILE_SLOTS * T::ES;                // omega tile plane
  double rowc[2] = {0.0, 0.0};
  for (int rd = 0; rd < rounds; ++rd) {
    const int64_t g = (chain * rounds + rd) * CW + wave;
    uint32_t raw[N];
    double v[2][N];  // [0] omega row (y[2k]), [1] psi row (y[2k+1])
    axisym_group<N, MODE>(mapP, GP, u, g, lane, j, in_wave, LP, LO, D, w, wj, ns, raw, v[0],
                          v[1]);
    SeamOut so;
    if constexpr (SEAM) so.base = sp.buf + sp.colour[chain] * sp.n_node * 2;
    chain_emit<N, 2, false, CW, SEAM>(y, raw, v, lane, wave, rd, in_wave, carry, rowc, accumulate,
                                      sp.round_sync, nullptr, so);
  }
}

// ---------------------------------------------------------------------------
// Poisson stiffness action on the fp64 matrix cores (n = p + 1 <= 16).
//
// One element per wavefront, its nodal arrays held as 16 x 16 tiles (zero
// padded) in the v_mfma_f64_16x16x4_f64 accumulator layout: lane l, register
// i holds entry (row h + 4i, column c) with c = l & 15, h = l >> 4 ("L1":
// lane <-> xi1 index j, registers <-> xi0 index m).  Register i is also the
// B operand of k-step i of a product contracting over the row index, and
// used as the A operand it supplies the TRANSPOSED tile.  With A = D held as
// Da[s] = D[c][4s + h] and Dt[s] = D[4s + h][c]:
//   d0 = D U     = mfma(Da, U_L1)        d1 = U D^T = mfma(U_L2, Da)
//   w0 = G00 d0 + G01 d1,  w1 = G01 d0 + G11 d1      (pointwise, L1)
//   y  = D^T w0 + w1 D = mfma(Dt, w0) + mfma(w1_L2, Dt)
// where X_L2 (lane <-> m, registers <-> j) is X transposed through a
// wave-private 16 x 17 LDS tile (rows padded to 17 doubles: the row write
// and the column read are both bank-conflict free).  4 products x ceil(n/4)
// MFMAs per element; map, u and the factors are read in the L1 layout only.
// One element per wavefront: walking 2 / 4 / 8 slots per wavefront with D
// kept in registers and the next map prefetched measured 10 / 24 / 36 %
// slower at p = 12 than more, shorter waves.  Same arithmetic as the column kernel (SURVEY.md §8(a)
// a11), summed in a different order.
//
// Padding lanes / rows (index >= n) load a valid entry (clamped index) and
// zero it with a select: no load sits under a branch.  Elements of one launch
// (colour) share no node (element-level colouring, build_plan_elem), so the
// scatter is plain stores / read-modify-writes.  Maps and factors are compact
// per element: mapP[slot][r][j], GP[slot][c][r][j].
//
// A first form (six products, U and the factors gathered in both layouts,
// no LDS) measured 0.215 / 0.179 ms at p = 12 / 15 against 0.191 / 0.139 for
// this one (profiles/r01/mfma_v1).
// ---------------------------------------------------------------------------
typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ dbl4 mfma_f64(double a, double b, dbl4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

constexpr int MFMA_EPB = BLOCK / WAVE;  // elements (waves) per workgroup

constexpr int MFMA_TS = 17;  // LDS tile row stride (doubles)

// transpose KS registers of a 16 x 16 C-layout tile through a wave-private
// LDS tile: out[i] (lane (h, c)) = in-tile entry (c, 4i + h)
template <int KS, int NT>
__device__ __forceinline__ void mfma_transpose(double* T, int h, int c, const double (*in)[KS],
                                               double (*out)[KS]) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < KS; ++i) T[t * 16 * MFMA_TS + (4 * i + h) * MFMA_TS + c] = in[t][i];
  wave_sync();
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < KS; ++i) out[t][i] = T[t * 16 * MFMA_TS + c * MFMA_TS + 4 * i + h];
  wave_sync();
}

#ifndef SEM_MFMA_MIN_WAVES
#define SEM_MFMA_MIN_WAVES 1
#endif
// B = 16 / n elements per tile side: for n <= 8 a wavefront packs B x B
// elements block-diagonally into one tile (D_blk = diag(D, ..., D) keeps the
// contractions inside each element), so (B n / 16)^2 of the tile is used
// instead of (n / 16)^2.  NODAL: the factors are re-derived per node from
// x_phys per global node, as in the column kernel, with the
// four Jacobian entries from four more products on coordinates taken
// relative to the element's node (0, 0).
template <int N, bool NODAL>
__global__ void __launch_bounds__(BLOCK, SEM_MFMA_MIN_WAVES)
    k_poisson_mfma(const uint32_t* __restrict__ mapP, const double* __restrict__ GP,
                   const double2* __restrict__ XG, const double* __restrict__ u,
                   double* __restrict__ y, const double* __restrict__ gD, const WVec<N> w,
                   int64_t s0, int64_t s1, int accumulate) {
  static_assert(N <= 16, "one 16x16 tile per element");
  constexpr int B = 16 / N;     // elements per tile side
  constexpr int TN = B * N;     // used rows / columns
  constexpr int EPT = B * B;    // elements per tile = per wavefront
  constexpr int KS = (TN + 3) / 4;  // k-steps covering the used rows
  constexpr int NN = N * N;
  __shared__ double lds[MFMA_EPB][(NODAL ? 2 : 1) * 16 * MFMA_TS];
  const int lane = threadIdx.x % WAVE;
  const int wave = threadIdx.x / WAVE;
  const int64_t slot0 = s0 + ((int64_t)blockIdx.x * MFMA_EPB + wave) * EPT;
  if (slot0 >= s1) return;  // uniform per wavefront; no workgroup barrier below
  double* T = lds[wave];
  const int c = lane & 15;
  const int h = lane >> 4;
  const bool cok = c < TN;
  const int cl = cok ? c % N : N - 1;  // local column of the lane's element
  const int ce = cok ? c / N : 0;      // element column inside the tile
  bool ok[KS];
  int off[KS];     // local (row, column) offset in an element's [n][n] arrays
  int64_t es[KS];  // slot of the element holding register i
  int rl[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    const int r = 4 * i + h;
    const bool rok = r < TN;
    rl[i] = rok ? r % N : N - 1;
    const int64_t sl = slot0 + (rok ? r / N : 0) * B + ce;
    ok[i] = cok && rok && sl < s1;
    es[i] = ok[i] ? sl : slot0;
    off[i] = rl[i] * N + cl;
  }
  double Da[KS], Dt[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + h;
    const bool same = cok && k < TN && k / N == ce;  // block-diagonal D
    const double a = gD[cl * N + k % N], t = gD[(k % N) * N + cl];
    Da[s] = same ? a : 0.0;
    Dt[s] = same ? t : 0.0;
  }
  uint32_t e[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) e[i] = mapP[es[i] * NN + off[i]];
  const dbl4 z = {0.0, 0.0, 0.0, 0.0};
  double g0[KS], g1[KS], g2[KS];
  if constexpr (NODAL) {
    const double wc = pick<N>(w, cl);
    double X[2][KS], XT[2][KS];
#pragma unroll
    for (int i = 0; i < KS; ++i) {
      const double2 xg = XG[e[i] & GID_MASK];
      const double2 x0 = XG[mapP[es[i] * NN] & GID_MASK];  // element's node (0, 0)
      X[0][i] = ok[i] ? xg.x - x0.x : 0.0;
      X[1][i] = ok[i] ? xg.y - x0.y : 0.0;
    }
    mfma_transpose<KS, 2>(T, h, c, X, XT);
    dbl4 jr0 = z, jr1 = z, js0 = z, js1 = z;  // dx/dr, dy/dr, dx/ds, dy/ds
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      jr0 = mfma_f64(Da[s], X[0][s], jr0);
      jr1 = mfma_f64(Da[s], X[1][s], jr1);
      js0 = mfma_f64(XT[0][s], Da[s], js0);
      js1 = mfma_f64(XT[1][s], Da[s], js1);
    }
#pragma unroll
    for (int i = 0; i < KS; ++i) {
      const double det = jr0[i] * js1[i] - js0[i] * jr1[i];
      const double sc = ok[i] ? (pick<N>(w, rl[i]) * wc) * fast_rcp(det) : 0.0;
      g0[i] = sc * fma(js1[i], js1[i], js0[i] * js0[i]);
      g1[i] = -sc * fma(js1[i], jr1[i], js0[i] * jr0[i]);
      g2[i] = sc * fma(jr1[i], jr1[i], jr0[i] * jr0[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < KS; ++i) {
      const double* gp = GP + es[i] * (3 * NN) + off[i];
      g0[i] = gp[0 * NN];
      g1[i] = gp[1 * NN];
      g2[i] = gp[2 * NN];
    }
  }
  double U[1][KS], UT[1][KS];
  uint32_t raw[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    const double v = u[e[i] & GID_MASK];
    U[0][i] = ok[i] ? v : 0.0;
    raw[i] = ok[i] ? e[i] : (W_SKIP << CODE_SHIFT);
  }
  mfma_transpose<KS, 1>(T, h, c, U, UT);
  dbl4 d0 = z, d1 = z;
#pragma unroll
  for (int s = 0; s < KS; ++s) d0 = mfma_f64(Da[s], U[0][s], d0);
#pragma unroll
  for (int s = 0; s < KS; ++s) d1 = mfma_f64(UT[0][s], Da[s], d1);
  double w0[KS], W1[1][KS], W1T[1][KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    w0[i] = ok[i] ? fma(g0[i], d0[i], g1[i] * d1[i]) : 0.0;
    W1[0][i] = ok[i] ? fma(g1[i], d0[i], g2[i] * d1[i]) : 0.0;
  }
  mfma_transpose<KS, 1>(T, h, c, W1, W1T);
  dbl4 acc = z;
#pragma unroll
  for (int s = 0; s < KS; ++s) acc = mfma_f64(Dt[s], w0[s], acc);
#pragma unroll
  for (int s = 0; s < KS; ++s) acc = mfma_f64(W1T[0][s], Dt[s], acc);
  // row 4i + h < TN implies i < KS; padding entries carry SKIP
#pragma unroll
  for (int i = 0; i < KS; ++i) emit1<false>(y, raw[i], acc[i], accumulate);
}

// ---------------------------------------------------------------------------
// Poisson stiffness action on the fp64 matrix cores for n = 17 (p = 16),
// where one element no longer fits a 16 x 16 tile.
//
// The contraction along one index is a GEMM whose N dimension is the other
// index: d0[:, j] = D U[:, j] for every line j of every element.  A pair of
// wavefronts takes EW = 3 elements and flattens their lines, f = 17 e + l,
// into T = 4 N-tiles of 16 (51 of 64 used, the column kernel's lane use),
// two tiles per wavefront.  The output and contraction index (17) is folded
// by the centro-antisymmetry of D (D[16-m][16-r] = -D[m][r]): with
// ua_a = x_a - x_{16-a}, us_a = x_a + x_{16-a} (a < 8),
//   s'_m = sum_a (D[m][a] - D[m][16-a]) / 2 ua_a      (m < 8),   out[8] = sum_a D[8][a] ua_a
//   t'_m = sum_a (D[m][a] + D[m][16-a]) / 2 us_a + D[m][8] x_8
//   out[m] = s'_m + t'_m,  out[16-m] = s'_m - t'_m
// i.e. one accumulator over K = ua (2 k-steps: s' rows 0..7 and out[8] in
// row 8) and one over K = us plus x_8 (3 k-steps: t' rows 0..7): 5 MFMAs per
// tile and contraction instead of 2 x 5 for the unfolded 17 x 17.  Lane
// (h = lane >> 4, c = lane & 15) of tile t holds line f = 16 t + c at the
// entries a = h, 4 + h, 16 - h, 12 - h (+ 8 for h = 0): exactly the B
// operands it supplies, and -- C row = h + 4 i -- exactly the outputs it
// receives, so a contraction maps a lane's five entries to the same five
// entries.  The same code contracts along the other index when the lines
// are the element's rows ("Y" layout) instead of its columns ("X").
//
//   d0 = D U (X),  d1 = U D^T (Y),  w0/w1 pointwise (X),
//   y = D^T w0 (X) + w1 D (Y)
//
// X <-> Y go through the pair's [3][17][17] LDS plane, updated in place (in
// each phase a lane writes back exactly the entries it read), with a
// workgroup barrier between phases.  Elements of one launch share no node
// (element colouring, build_plan_elem); stored factors per element slot as
// for k_poisson_mfma.  The scatter reads its read-modify-write operands for
// all of a lane's entries at once, before the last contraction (predicated
// buffer loads as in rmw_prefetch); a branch around a load and its store per
// entry serialised the round trips (first form: 68 us per colour launch at
// p = 16, 198^2, against 0.16 ms per action for the column kernel).
// ---------------------------------------------------------------------------
constexpr int MF17_N = 17;
constexpr int MF17_EW = 3;                          // elements per wavefront pair
constexpr int MF17_TW = 2;                          // N-tiles per wavefront (4 per pair)
constexpr int MF17_PAIRS = BLOCK / (2 * WAVE);      // wavefront pairs per workgroup
constexpr int MF17_PLANE = MF17_EW * 17 * 17 + 2 * WAVE;  // doubles per pair plane (+ junk)

// A operands of one centro-antisymmetric 17 x 17 matrix M (lane row rho =
// lane & 15, k = lane >> 4): s-steps, t-steps, the x_8 step
struct MF17A {
  double s0, s1, t0, t1, m;
};

__device__ __forceinline__ MF17A mf17_operands(const double* __restrict__ gD, bool tr, int lane) {
  const int rho = lane & 15, q = lane >> 4;
  auto M = [&](int i, int j) { return tr ? gD[j * MF17_N + i] : gD[i * MF17_N + j]; };
  MF17A A;
  const int rr = rho < 8 ? rho : 0;
  const double s0 = 0.5 * (M(rr, q) - M(rr, 16 - q)), s1 = 0.5 * (M(rr, 4 + q) - M(rr, 12 - q));
  const double t0 = 0.5 * (M(rr, q) + M(rr, 16 - q)), t1 = 0.5 * (M(rr, 4 + q) + M(rr, 12 - q));
  const double m8a = M(8, q), m8b = M(8, 4 + q), mm = M(rr, 8);
  A.s0 = rho < 8 ? s0 : (rho == 8 ? m8a : 0.0);
  A.s1 = rho < 8 ? s1 : (rho == 8 ? m8b : 0.0);
  A.t0 = rho < 8 ? t0 : 0.0;
  A.t1 = rho < 8 ? t1 : 0.0;
  A.m = (rho < 8 && q == 0) ? mm : 0.0;
  return A;
}

// v[0..4] = line entries a = h, 4 + h, 16 - h, 12 - h, 8 (v[4] zero unless
// h = 0) -> the same entries of M times the line
__device__ __forceinline__ void mf17_contract(const MF17A& A, double (&v)[5]) {
  const dbl4 z = {0.0, 0.0, 0.0, 0.0};
  const double ua0 = v[0] - v[2], ua1 = v[1] - v[3];
  const double us0 = v[0] + v[2], us1 = v[1] + v[3];
  dbl4 as = mfma_f64(A.s0, ua0, z);
  dbl4 at = mfma_f64(A.t0, us0, z);
  as = mfma_f64(A.s1, ua1, as);
  at = mfma_f64(A.t1, us1, at);
  at = mfma_f64(A.m, v[4], at);
  v[0] = as[0] + at[0];
  v[2] = as[0] - at[0];
  v[1] = as[1] + at[1];
  v[3] = as[1] - at[1];
  v[4] = as[2];  // row 8 + h: out[8] for h = 0, zero rows otherwise
}

// Persistent form: a grid of resident workgroups, each wavefront pair walks
// element triples q = pair, pair + P, ... (P pairs in the grid) and reads
// the NEXT triple's map (during phase B) and u (during phase C) while the
// current one computes, and the current triple's factors before phase A:
// the per-triple chain map -> gather -> factors is off the critical path
// except for the first triple of each pair.  240 VGPRs, 2 waves/SIMD, no
// scratch.  p = 16, 198^2, two runs alternating on one box
// (profiles/r03/mfma17/persist/, median kernel ms per action): 0.180 /
// 0.182 against 0.185 / 0.187 for the earlier form with one wavefront pair
// per triple (factors read before phase B; reading them in phase C at 3
// waves/SIMD 0.195 / 0.199, 4 waves with scratch 0.197, profiles/r03/
// mfma17/); the column kernel 0.159 / 0.160 on that box -- the gain is
// small, so the per-triple chain is not what bounds the kernel (DESIGN.md
// §4.6).  The one-pair-per-triple form was removed after these runs.
#ifndef SEM_MF17P_WAVES
#define SEM_MF17P_WAVES 2
#endif
template <int N, bool SEAM>
__global__ void __launch_bounds__(BLOCK, SEM_MF17P_WAVES)
    k_poisson_mfma17p(const uint32_t* __restrict__ mapP, const double* __restrict__ GP,
                      const double* __restrict__ u, double* __restrict__ y,
                      const double* __restrict__ gD, int64_t s0, int64_t s1, int accumulate,
                      SeamPlan sp) {
  static_assert(N == MF17_N, "folded multi-element form of n = 17");
  constexpr int NN = N * N, T = MF17_TW;
  __shared__ double lds[MF17_PAIRS][MF17_PLANE];
  const int lane = threadIdx.x % WAVE;
  const int wave = threadIdx.x / WAVE;
  const int pair = wave >> 1, half = wave & 1;
  const int64_t ntr = (s1 - s0 + MF17_EW - 1) / MF17_EW;  // element triples
  const int64_t np = (int64_t)gridDim.x * MF17_PAIRS;
  const int64_t q0 = (int64_t)blockIdx.x * MF17_PAIRS;  // the workgroup's first pair
  // every pair of a workgroup runs the first pair's iteration count (the
  // workgroup barriers); a pair past the end works on slot s0, writes nothing
  const int64_t iters = q0 < ntr ? (ntr - q0 + np - 1) / np : 0;
  double* P = lds[pair];
  const int h = lane >> 4, c = lane & 15;
  const bool hm = h == 0;  // owner of the middle entry
  const int R[5] = {h, 4 + h, 16 - h, 12 - h, 8};
  const MF17A AD = mf17_operands(gD, false, lane);
  const MF17A AT = mf17_operands(gD, true, lane);
  constexpr int JUNK = MF17_EW * NN;
  int ef[T], lf[T];  // element and line of tile 2 half + t
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int f = 16 * (2 * half + t) + c;
    ef[t] = f / N;
    lf[t] = f - ef[t] * N;
  }
  // triple q: base slot, per-tile validity and the element used (0 stands in)
  auto base = [&](int64_t q) { return q < ntr ? s0 + q * MF17_EW : s0; };
  auto valid = [&](int64_t q, int t) {
    return q < ntr && ef[t] < MF17_EW && s0 + q * MF17_EW + ef[t] < s1;
  };
  auto go = [&](int t, int el, int k) { return el * NN + lf[t] + (k < 4 || hm ? R[k] : 0) * N; };

  int64_t q = q0 + pair;
  uint32_t raw[T][5];
  double uv[T][5];
  {
    const int64_t sb = base(q);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int el = valid(q, t) ? ef[t] : 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) raw[t][k] = mapP[sb * NN + go(t, el, k)];
    }
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int k = 0; k < 5; ++k) uv[t][k] = u[raw[t][k] & GID_MASK];
  }
  for (int64_t it = 0; it < iters; ++it, q += np) {
    const int64_t sb = base(q), qn = q + np, sbn = base(qn);
    bool ok[T];
    int el[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      ok[t] = valid(q, t);
      el[t] = ok[t] ? ef[t] : 0;
    }
    auto live = [&](int t, int k) { return ok[t] && (k < 4 || hm); };
    auto xo = [&](int t, int k) {
      return live(t, k) ? el[t] * NN + lf[t] + R[k] * N : JUNK + half * WAVE + lane;
    };
    auto yo = [&](int t, int k) {
      return live(t, k) ? el[t] * NN + lf[t] * N + R[k] : JUNK + half * WAVE + lane;
    };
    // factors of this triple
    double g[T][5][3];
    {
      const double* gq = GP + sb * (3 * NN);
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const double* gp = gq + go(t, el[t], k) + el[t] * (2 * NN);  // slot stride 3 NN
          g[t][k][0] = gp[0];
          g[t][k][1] = gp[NN];
          g[t][k][2] = gp[2 * NN];
        }
    }
    // phase A: U (X) into the plane, d0 = D U
    double d0[T][5];
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        d0[t][k] = live(t, k) ? uv[t][k] : 0.0;
        raw[t][k] = live(t, k) ? raw[t][k] : (W_SKIP << CODE_SHIFT);
        P[xo(t, k)] = d0[t][k];
      }
      mf17_contract(AD, d0[t]);
    }
    __syncthreads();
    // next triple's map
    uint32_t rawn[T][5];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int eln = valid(qn, t) ? ef[t] : 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) rawn[t][k] = mapP[sbn * NN + go(t, eln, k)];
    }
    // phase B: d1 = U D^T along the rows (Y), in place
#pragma unroll
    for (int t = 0; t < T; ++t) {
      double v[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) v[k] = live(t, k) ? P[yo(t, k)] : 0.0;
      mf17_contract(AD, v);
#pragma unroll
      for (int k = 0; k < 5; ++k) P[yo(t, k)] = v[k];
    }
    __syncthreads();
    // next triple's u
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int k = 0; k < 5; ++k) uv[t][k] = u[rawn[t][k] & GID_MASK];
    // phase C: w0 = G00 d0 + G01 d1 -> y0 = D^T w0, w1 = G01 d0 + G11 d1 in place
    double y0[T][5];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      double w1[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const double d1 = P[xo(t, k)];
        y0[t][k] = live(t, k) ? fma(g[t][k][0], d0[t][k], g[t][k][1] * d1) : 0.0;
        w1[k] = live(t, k) ? fma(g[t][k][1], d0[t][k], g[t][k][2] * d1) : 0.0;
      }
      mf17_contract(AT, y0[t]);
#pragma unroll
      for (int k = 0; k < 5; ++k) P[xo(t, k)] = w1[k];
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t ry = y_rsrc(y);
    double prev[T][5];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const uint32_t a = (raw[t][k] >> CODE_SHIFT) & 3u;
        const bool need = a == W_RMW || (a == W_STORE && accumulate);
        const uint32_t off = need ? (raw[t][k] & GID_MASK) * 8u : 0x80000000u;
        prev[t][k] =
            __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(ry, off, 0, CPOL_NT));
      }
    // phase D: y1 = w1 D along the rows (Y), in place
#pragma unroll
    for (int t = 0; t < T; ++t) {
      double v[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) v[k] = live(t, k) ? P[yo(t, k)] : 0.0;
      mf17_contract(AT, v);
#pragma unroll
      for (int k = 0; k < 5; ++k) P[yo(t, k)] = v[k];
    }
    __syncthreads();
    // phase E: y = y0 + y1 (X), scatter (a lane reads only its own plane
    // entries here and writes only those in the next phase A: no barrier)
#pragma unroll
    for (int t = 0; t < T; ++t) {
      double* sbase = nullptr;
      if constexpr (SEAM) sbase = sp.buf + (int64_t)sp.colour[sb + el[t]] * sp.n_node;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const uint32_t a = (raw[t][k] >> CODE_SHIFT) & 3u;
        const uint32_t gid = raw[t][k] & GID_MASK;
        const double v = y0[t][k] + P[xo(t, k)];
        if (a == W_STORE || a == W_RMW) {
          y[gid] = prev[t][k] + v;
        } else if (a == W_ATOMIC) {
          if constexpr (SEAM)
            sbase[gid] = v;
          else
            atomic_add_f64(y + gid, v);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int k = 0; k < 5; ++k) raw[t][k] = rawn[t][k];
  }
}

// ---------------------------------------------------------------------------
// Geometry: nodes -> x_phys -> J -> det/inv -> W -> operator factors.
// Thread per local node, EPB elements per block, LDS staging (setup path).
// ---------------------------------------------------------------------------
template <int N>
struct GeomShape {
  static constexpr int NN = N * N;
  static constexpr int EPB = (NN >= 256) ? 1 : 256 / NN;
  static constexpr int THREADS = ((EPB * NN + 63) / 64) * 64;
};

// Error-free transformations for the compensated equispaced->GLL transform:
// a*b = p + e exactly, a + b = s + e exactly (round to nearest, no fast-math).
// Contraction is off inside them: hipcc's default -ffp-contract=fast would
// otherwise fuse the rounded product p of two_prod into the following
// two_sum's addition (s = s' + a*b as one fma), so that s no longer adds the
// p whose error e describes and the compensation is silently lost (the
// hexahedral p = 14 geometry measured exactly the plain-float64 error,
// 1.34e-10 of the action against the extended-precision oracle).
__device__ __forceinline__ void two_prod(double a, double b, double& p, double& e) {
#pragma clang fp contract(off)
  p = a * b;
  e = fma(a, b, -p);
}
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
#pragma clang fp contract(off)
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}
// s_hi + s_lo ~= s_hi_in + sum_i a[i*sa] * (bh[i*sb] + bl[i*sb]) to about twice
// the working precision (Ogita-Rump-Oishi Dot2; the lo parts enter plainly).
template <int N>
__device__ __forceinline__ void dot2(const double* a, int sa, const double* bh, const double* bl,
                                     int sb, double& hi, double& lo) {
  double s = 0.0, c = 0.0;
  for (int i = 0; i < N; ++i) {
    double p, ep, es;
    two_prod(a[i * sa], bh[i * sb], p, ep);
    two_sum(s, p, s, es);
    c += ep + es;
    if (bl) c = fma(a[i * sa], bl[i * sb], c);
  }
  hi = s + c;
  lo = c - (hi - s);
}

template <int N>
__global__ void __launch_bounds__(GeomShape<N>::THREADS)
    k_geometry(const double* __restrict__ nodes, int64_t n_node, const uint32_t* __restrict__ e2n,
               int64_t n_elem, const double* __restrict__ gVinv, const double* __restrict__ gD,
               const double* __restrict__ gw, int op_kind, int epw, const int* __restrict__ epos,
               double* __restrict__ GP, double* __restrict__ xph, double* __restrict__ Jo,
               double* __restrict__ iJo, double* __restrict__ dJo, double* __restrict__ dJW,
               double2* __restrict__ XG, const uint32_t* __restrict__ owner,
               const double2* __restrict__ XGin, const double* __restrict__ XEin,
               unsigned long long* __restrict__ n_bad) {
  using S = GeomShape<N>;
  constexpr int NN = S::NN;
  constexpr int EPB = S::EPB;
  const int LW = epw * N;  // packed row: the epw elements of a group (1 for the MFMA kernel)
  __shared__ double sV[NN], sD[NN], sw[N];
  __shared__ double sx[EPB][2][NN], st[EPB][2][NN], stl[EPB][2][NN];
  const int tid = threadIdx.x;
  for (int i = tid; i < NN; i += blockDim.x) {
    sV[i] = gVinv[i];
    sD[i] = gD[i];
  }
  if (tid < N) sw[tid] = gw[tid];
  const int el = tid / NN;
  const int node = tid - el * NN;
  const int m = node / N;
  const int nq = node - m * N;
  const int64_t e = (int64_t)blockIdx.x * EPB + el;
  const bool act = (el < EPB) && (e < n_elem);
  uint32_t gi = 0;
  if (act) {
    gi = e2n[e * NN + node];
    if (XEin) {  // x_phys given per element (sem_geom_from_xphys)
      sx[el][0][node] = XEin[(e * 2 + 0) * NN + node];
      sx[el][1][node] = XEin[(e * 2 + 1) * NN + node];
    } else if (XGin) {  // x_phys already known per global node (NODAL mode re-derivation)
      const double2 xg = XGin[gi];
      sx[el][0][node] = xg.x;
      sx[el][1][node] = xg.y;
    } else {
      sx[el][0][node] = nodes[gi];
      sx[el][1][node] = nodes[n_node + gi];
    }
  }
  __syncthreads();
  // x_phys = Vinv X Vinv^T   (compute_coeffs_grid_eq: dim 0 then dim 1),
  // evaluated on coordinates relative to the element's node (0,0): the map
  // is translation invariant (V_eq reproduces constants) and J = D x_phys
  // then no longer cancels the O(1) offset against O(h) variations.
  // Both passes are compensated dot products (dot2, the intermediate kept as
  // hi + lo) on the exact relative coordinates (two_sum): Vinv has entries
  // up to ~170 at p = 16 (cond(V_eq) ~ 1e5), and J = D x_phys amplifies the
  // rounding of plain float64 sums by ~n^2/4; cfg4 p = 16 on the device:
  // 4.9e-11 -> 2.9e-12 rel-L2 of the action against the extended-precision
  // oracle (the rounds 3-5 passes had their compensation
  // fused away by contraction, see two_prod).
  double x0[2] = {0.0, 0.0};
  const bool given = XGin || XEin;  // x_phys given: no transform
  if (act && !given) {
    x0[0] = sx[el][0][0];
    x0[1] = sx[el][1][0];
    for (int c = 0; c < 2; ++c) {
      // the exact difference hi + lo (two_sum): the rounding of a float64
      // difference alone is amplified by cond(V_eq)
      double xr[N], xrl[N];
      for (int i = 0; i < N; ++i) two_sum(sx[el][c][i * N + nq], -x0[c], xr[i], xrl[i]);
      double hi, lo;
      dot2<N>(&sV[m * N], 1, xr, xrl, 1, hi, lo);
      st[el][c][node] = hi;
      stl[el][c][node] = lo;
    }
  }
  __syncthreads();
  double xp[2] = {0.0, 0.0};
  if (act && given) {
    x0[0] = sx[el][0][0];
    x0[1] = sx[el][1][0];
    xp[0] = sx[el][0][node] - x0[0];
    xp[1] = sx[el][1][node] - x0[1];
  } else if (act) {
    for (int c = 0; c < 2; ++c) {
      double hi, lo;
      dot2<N>(&sV[nq * N], 1, &st[el][c][m * N], &stl[el][c][m * N], 1, hi, lo);
      xp[c] = hi;
    }
  }
  __syncthreads();
  if (act) {
    sx[el][0][node] = xp[0];
    sx[el][1][node] = xp[1];
  }
  __syncthreads();
  if (!act) return;
  // J[c][d] = d x_c / d xi_d (TensorProduct.gradient, swapaxes(0,1))
  double J[2][2];
  for (int c = 0; c < 2; ++c) {
    double a = 0.0, b = 0.0;
    for (int r = 0; r < N; ++r) {
      a = fma(sD[m * N + r], sx[el][c][r * N + nq], a);
      b = fma(sD[nq * N + r], sx[el][c][m * N + r], b);
    }
    J[c][0] = a;
    J[c][1] = b;
  }
  // det_inv_2x2 (sem/linalg.py:105-115)
  const double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
  const double rdet = 1.0 / det;
  const double iJ00 = J[1][1] * rdet, iJ01 = -J[0][1] * rdet;
  const double iJ10 = -J[1][0] * rdet, iJ11 = J[0][0] * rdet;
  // detJxW via TensorQuadratureRule.xweight (sem/quadratures.py:268-275)
  const double W = det * sw[m] * sw[nq];
  if (!(det > 0.0)) atomicAdd(n_bad, 1ull);
  const int64_t base = e * NN + node;
  const double xabs0 = xp[0] + x0[0];
  const double xabs1 = xp[1] + x0[1];
  // x_phys per global node, written by the node's first element only (the
  // copies of a shared node differ in rounding; one writer keeps it
  // deterministic)
  if (XG && owner[gi] == (uint32_t)e) XG[gi] = make_double2(xabs0, xabs1);
  if (xph) {
    xph[(e * 2 + 0) * NN + node] = xabs0;
    xph[(e * 2 + 1) * NN + node] = xabs1;
  }
  if (Jo) {
    Jo[(e * 4 + 0) * NN + node] = J[0][0];
    Jo[(e * 4 + 1) * NN + node] = J[0][1];
    Jo[(e * 4 + 2) * NN + node] = J[1][0];
    Jo[(e * 4 + 3) * NN + node] = J[1][1];
  }
  if (iJo) {
    iJo[(e * 4 + 0) * NN + node] = iJ00;
    iJo[(e * 4 + 1) * NN + node] = iJ01;
    iJo[(e * 4 + 2) * NN + node] = iJ10;
    iJo[(e * 4 + 3) * NN + node] = iJ11;
  }
  if (dJo) dJo[base] = det;
  if (dJW) dJW[base] = W;
  if (GP) {
    const int64_t pos = epos[e];  // packed position slot * epw + lane element
    const int64_t gg = pos / epw;
    const int kk = (int)(pos - gg * epw);
    const int ncomp = (op_kind == 0) ? 3 : (op_kind == 1 ? 7 : 9);
    double* o = GP + gg * (int64_t)(ncomp * N * LW) + m * LW + kk * N + nq;
    const double A00 = iJ00 * iJ00 + iJ01 * iJ01;
    const double A01 = iJ00 * iJ10 + iJ01 * iJ11;
    const double A11 = iJ10 * iJ10 + iJ11 * iJ11;
    if (op_kind == 0) {
      o[0 * N * LW] = W * A00;
      o[1 * N * LW] = W * A01;
      o[2 * N * LW] = W * A11;
    } else {
      const double rho = xabs0;
      const double rW = rho * W;
      o[0 * N * LW] = rW * A00;
      o[1 * N * LW] = rW * A01;
      o[2 * N * LW] = rW * A11;
      o[3 * N * LW] = 2.0 * W * iJ00;
      o[4 * N * LW] = 2.0 * W * iJ10;
      o[5 * N * LW] = W / rho;
      o[6 * N * LW] = rW * rho;
      if (ncomp == 9) {  // Navier-Stokes advection: (W/rho) iJ01, (W/rho) iJ11
        o[7 * N * LW] = (W / rho) * iJ01;
        o[8 * N * LW] = (W / rho) * iJ11;
      }
    }
  }
}

}  // namespace semk
