// Hexahedral (3-D) kernels of libsem_hip.so (included by sem_hex.hip only).
//
// The reference's tensor-product layer is N-dimensional: TensorProduct.deriv
// / gradient apply D along any axis of an [..., n, n, n] coefficient array
// (sem/basis_functions.py:626-650), compute_coeffs_grid_eq solves V_eq along
// each axis (:599-624) and TensorQuadratureRule.xweight multiplies by the
// tensor weights (sem/quadratures.py:268-275); only the 2x2 Jacobian inverse
// (sem/mapping.py:110-111) and the quad-only example stop it at 2-D.  These
// kernels run the same per-element algebra on hexahedra: local node (a, b, c)
// <-> (xi0, xi1, xi2), C-contiguous, xi2 fastest, as the reference lays out
// an [n, n, n] coefficient block.
//
//   u_e = u[map[e]]                                      (gather)
//   d_k = D along xi_k of u_e,  k = 0, 1, 2              (D(x)I(x)I, I(x)D(x)I, I(x)I(x)D)
//   w_k = sum_l G_kl d_l,  G = detJxW invJ invJ^T        (6 factors per node)
//   y_e = sum_k D^T along xi_k of w_k                    (transposed pass)
//   y[map[e]] += y_e                                     (scatter, no atomics)
//
// CDNA4 mapping:
//  * one element = an n x n tile of threads, thread (b, c) owns the element
//    COLUMN of nodes (0..n-1, b, c) along xi0 in registers; a 256-thread
//    workgroup holds S = floor(256 / n^2) such tiles ("slots").  The xi0
//    contractions run in registers; the xi1 / xi2 ones read the other
//    threads' columns from LDS (three n^3 buffers per slot: u, w1, w2, so an
//    element costs two workgroup barriers).
//  * each slot walks a CHAIN of elements along xi0 (consecutive elements of a
//    chain share their xi0 face with identical (b, c) ordering): the node row
//    a = n-1 of one element IS row a = 0 of the next, held by the same
//    thread, so that face is summed in a register and written once.
//  * every other node shared by several writers (element edges / faces
//    between chains, chain ends) is written into a per-writer SLOT and summed
//    in a fixed order by a second launch (k_hex_seam_sum): deterministic, no
//    atomics; nodes with one writer are plain stores.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace semh {

constexpr int HEX_MIN_N = 2;
constexpr int HEX_MAX_N = 17;  // p <= 16

// element slots per workgroup: as many n x n thread tiles as fit in 256 threads
constexpr int hex_slots(int n) { return 256 / (n * n) > 0 ? 256 / (n * n) : 1; }
constexpr int hex_threads(int n) { return (hex_slots(n) * n * n + 63) / 64 * 64; }
// boundary columns of an element: b or c on the element boundary
constexpr int hex_nbc(int n) { return 4 * (n - 1); }

// launch tables of the hex plan (device pointers; sem_hex.hip builds them)
struct HexLaunch {
  const int* wg_off;                // [n_wg] first launch position of workgroup w
  const int* wg_len;                // [n_wg] chain length of workgroup w
  const int* elist;                 // [pos] element at position wg_off + k*S + s, -1 = empty slot
  const unsigned long long* cmask;  // [pos] boundary columns written into slots
  const uint8_t* cflag;             // [n_wg*S] bit 0: chain head face slotted, bit 1: tail face,
                                    // bit 2: the sub-chain's xi2 = 0 face is the xi2 = n-1
                                    // face of slot s-1's (z-merge: summed in LDS)
  double* slot;                     // column slots [pos][n][NBC], then face slots [n_wg*S][2][n^2]
  int64_t face_base;
  // template map (the TM kernels): every element's node ids are its first
  // node's id + one shared offset block -- a structured numbering -- so a
  // thread keeps its column's n offsets in registers and reads one base per
  // element instead of n map entries
  const uint32_t* ebase = nullptr;  // [E] node id of local node (0, 0, 0)
  const int* tmpl = nullptr;        // [n^3] offsets
};

enum { HEX_SET = 0, HEX_ACC = 1, HEX_DIAG = 2 };

// z-merge (xi2 faces between the slots of a workgroup summed in LDS, one
// writer fewer per merged node) in the three-block kernel: the exchange
// goes through its w1 block (no LDS of its own); the plan decides at run
// time (SEM_HEX_ZMERGE=0 in the environment turns it off); building with
// -DSEM_HEX_ZMERGE=0 removes the code
#ifndef SEM_HEX_ZMERGE
#define SEM_HEX_ZMERGE 1
#endif
constexpr bool HEX_ZMERGE = SEM_HEX_ZMERGE != 0;

// y-merge (three-block kernel, with the z-merge): the S slots of a
// workgroup form a Y x Z grid (Z = hex_grid_z(n) slots along xi2 per row, Y
// rows along xi1; Y = 1 when S is prime), and slot s hands its xi1 = 0 face
// to slot s - Z when that face IS slot s - Z's xi1 = n-1 face at every chain
// step (cflag bit 3, checked by the planner), through the w2 block.  Columns
// a slot already handed over in the z-merge (c = 0) stay out of the y-merge
// on both sides.  p = 1 / 2 / 3 / 4 / 7: 8 x 8, 4 x 7, 4 x 4, 2 x 5, 2 x 2
// slots; on by default at p <= 3 (sem_hex.hip ctx_init), SEM_HEX_YMERGE=1 / 0
// in the environment forces it.
constexpr int hex_grid_z(int n) {
  int z = hex_slots(n);
  for (int y = 2; y * y <= hex_slots(n); ++y)
    if (hex_slots(n) % y == 0) z = hex_slots(n) / y;
  return z;
}

// D as a kernel argument: the wave-uniform coefficients of the
// register-direction contractions (row a of D, for d0 = D u and y += D^T w0
// along xi0) are read with scalar loads (SGPR operands) instead of LDS
// broadcasts, which cost the LDS pipe as much as data reads.
template <int N>
struct HexD {
  double d[N * N];  // d[q*N + a] = D[q][a]: row q of D
};

// Layout of the stored factors (G00, G01, G02, G11, G12, G22 per element
// node) as three double2 pairs (00, 01), (02, 11), (12, 22).  SoA
// (HEX_GSOA, default): per element and node row a, three planes of n^2
// pairs, so one wave-instruction reads 64 lanes' pair j as one contiguous
// 1 KiB run; AoS (SEM_HEX_GSOA=0): the node's three pairs side by side
// (48 B per lane, each wave-instruction spread over 3 KiB).  Measured equal
// at p = 4..10 and 1.5 % faster at p = 2.  Either way a
// node row is 3 n^2 pairs.
#ifndef SEM_HEX_GSOA
#define SEM_HEX_GSOA 1
#endif
constexpr bool HEX_GSOA = SEM_HEX_GSOA != 0;
template <int N>
__host__ __device__ constexpr int64_t hex_g_off(int64_t e, int bc) {
  return e * (int64_t)N * N * N * 3 + (HEX_GSOA ? bc : 3 * bc);
}
template <int N>
__device__ __forceinline__ const double2* hex_g(const double* G, int64_t e, int bc) {
  return reinterpret_cast<const double2*>(G) + hex_g_off<N>(e, bc);
}

// boundary-column index of (b, c) in [0, 4(n-1)), -1 for an interior column
template <int N>
__device__ __forceinline__ int hex_bcol(int b, int c) {
  if (b == 0) return c;
  if (b == N - 1) return 3 * N - 4 + c;
  if (c == 0) return N + 2 * (b - 1);
  if (c == N - 1) return N + 2 * (b - 1) + 1;
  return -1;
}

// Poisson stiffness action on hexahedra (MODE HEX_SET / HEX_ACC), or the
// diagonal of the assembled operator (HEX_DIAG; u unused).  G: stored factors
// in the pair layout of hex_g (components 00, 01, 02, 11, 12, 22): a thread
// reads its node's six as three 16-byte loads.
#ifndef SEM_HEX_MIN_WAVES
#define SEM_HEX_MIN_WAVES 4
#endif
// occupancy request: above p = 10 the register arrays (column of u, y, the
// maps) exceed what four waves per SIMD allow, and one element slot per
// workgroup leaves LDS the limit anyway
constexpr int hex_min_waves(int n) { return n <= 11 ? SEM_HEX_MIN_WAVES : n <= 13 ? 2 : 1; }
template <int N, int MODE, bool TM = false>
__global__ void __launch_bounds__(hex_threads(N), hex_min_waves(N))
    k_hex_poisson(const double* __restrict__ u, double* __restrict__ y,
                  const uint32_t* __restrict__ map, const double* __restrict__ G,
                  const double* __restrict__ gD, HexLaunch P, const HexD<N> Dk) {
  constexpr int N2 = N * N, N3 = N2 * N, S = hex_slots(N), T = hex_threads(N), NBC = hex_nbc(N);
  constexpr int GROW = 3 * N2, GPAIR = HEX_GSOA ? N2 : 1;  // factor layout (hex_g)
  __shared__ double sD[N2];
  __shared__ double sU[S * N3];
  __shared__ double sA[S * N3];
  __shared__ double sB[S * N3];
  // z-merge: the xi2 = 0 face of slot s (s >= 1) handed to slot s-1 through
  // the w1 block, free once every thread has finished the transposed pass
  // (a buffer of its own, 1.3 KB at n = 9, took the workgroup one 512-byte
  // granule past three per CU: element kernel 225 -> 241 us)
  constexpr bool ZM = HEX_ZMERGE;
  const int tid = threadIdx.x;
  for (int i = tid; i < N2; i += T) sD[i] = gD[i];
  const int w = blockIdx.x;
  const int L = P.wg_len[w];
  const int base = P.wg_off[w];
  const int s = tid / N2;
  const int bc = tid - s * N2;
  const int b = bc / N, c = bc - b * N;
  const bool active = s < S && P.elist[base + s] >= 0;
  const int sl = active ? s : 0;
  double* const su = sU + sl * N3;
  double* const sa = sA + sl * N3;
  double* const sb = sB + sl * N3;
  const int bcol = hex_bcol<N>(b, c);
  const uint8_t cf = active ? P.cflag[w * S + s] : 0;
  // z-merge: slot s hands its xi2 = 0 face to slot s-1, whose xi2 = n-1 face
  // holds the same nodes in the same (a, b) order (the planner checked every
  // chain step); the merged node then has one writer fewer
  const bool give = (cf & 4) && c == 0;
  [[maybe_unused]] const bool take = active && c == N - 1 && s + 1 < S && (P.cflag[w * S + s + 1] & 4);
  // y-merge: slot s hands its xi1 = 0 face (b = 0) to slot s - GZ, except
  // the column it already handed over in the z-merge (or whose receiver did)
  constexpr int GZ = hex_grid_z(N);
  constexpr bool YM = ZM && GZ < S;
  [[maybe_unused]] bool ygive = false, ytake = false;
  if constexpr (YM) {
    ygive = (cf & 8) && b == 0 && s >= GZ &&
            !(c == 0 && ((cf & 4) || (P.cflag[w * S + s - GZ] & 4)));
    if (active && b == N - 1 && s + GZ < S) {
      const uint8_t cg = P.cflag[w * S + s + GZ];
      ytake = (cg & 8) && !(c == 0 && ((cg & 4) || (cf & 4)));
    }
  }
  [[maybe_unused]] bool wg_merge = false;
  if constexpr (ZM)
#pragma unroll
    for (int t = 1; t < S; ++t) wg_merge |= (P.cflag[w * S + t] & 12) != 0;
  double* const face = P.slot + P.face_base + (int64_t)(w * S + sl) * 2 * N2 + bc;
  __syncthreads();  // sD
  double carry = 0.0;
  // the element map of the next chain step is loaded one step ahead
  uint32_t mn[N];
  int en = active ? P.elist[base + s] : 0;
  [[maybe_unused]] int toff[TM ? N : 1];
  if constexpr (TM)
#pragma unroll
    for (int a = 0; a < N; ++a) toff[a] = P.tmpl[a * N2 + bc];
  if (active) {
    if constexpr (TM) {
      const uint32_t eb = P.ebase[en];
#pragma unroll
      for (int a = 0; a < N; ++a) mn[a] = eb + (uint32_t)toff[a];
    } else {
#pragma unroll
      for (int a = 0; a < N; ++a) mn[a] = map[(int64_t)en * N3 + a * N2 + bc];
    }
  }
#pragma unroll 1
  for (int k = 0; k < L; ++k) {
    const int pos = base + k * S + s;
    const int e = en;
    uint32_t m[N];
#pragma unroll
    for (int a = 0; a < N; ++a) m[a] = mn[a];
    const double2* g = hex_g<N>(G, e, bc);
    double uc[MODE != HEX_DIAG ? N : 1];
    if (active) {
      if constexpr (MODE != HEX_DIAG) {
#pragma unroll
        for (int a = 0; a < N; ++a) {
#ifdef SEM_HEX_DIAG_NOGATHER  // diagnostic builds only: no u gather
          uc[a] = (double)m[a];
#else
          uc[a] = u[m[a]];
#endif
        }
#pragma unroll
        for (int a = 0; a < N; ++a) su[a * N2 + bc] = uc[a];
      } else {
        // diagonal: G00 of this column, G11 / G22 of the other threads' nodes
#pragma unroll
        for (int a = 0; a < N; ++a) {
          su[a * N2 + bc] = g[a * GROW].x;              // G00
          sa[a * N2 + bc] = g[a * GROW + GPAIR].y;      // G11
          sb[a * N2 + bc] = g[a * GROW + 2 * GPAIR].y;  // G22
        }
      }
    }
    __syncthreads();
    if (active && k + 1 < L) {
      en = P.elist[pos + S];
      if constexpr (TM) {
        const uint32_t eb = P.ebase[en];
#pragma unroll
        for (int a = 0; a < N; ++a) mn[a] = eb + (uint32_t)toff[a];
      } else {
#pragma unroll
        for (int a = 0; a < N; ++a) mn[a] = map[(int64_t)en * N3 + a * N2 + bc];
      }
    }
    // The contractions run with the summation index outermost and NOT
    // unrolled, the node row a unrolled inside: every register array is
    // indexed by a compile-time a, and a step holds only its own operands
    // (a fully unrolled a x r nest lets the scheduler hoist the LDS and G
    // reads of later rows: 256+ VGPRs and spills from n = 6 on).
    double yv[N];
#pragma unroll
    for (int a = 0; a < N; ++a) yv[a] = 0.0;
    if constexpr (MODE != HEX_DIAG) {
      if (active) {
        // Node row a (outer, not unrolled): d = (D u)_a along xi0 / xi1 /
        // xi2, w = G d; w1 / w2 to LDS; y += D[a][.] w0, the D^T contraction
        // along xi0, in registers (D row a read once per row with scalar
        // loads: it serves both xi0 contractions).  w0 never goes through
        // LDS, and su is free for the next step's u after the barrier.
        // (The r-outer form with d0 / d1 / d2 arrays: 223.6 against
        // 218-220 us, profiles/r05/hex/a_outer/.)
#pragma unroll 1
        for (int a = 0; a < N; ++a) {
          double d0 = 0.0, d1 = 0.0, d2 = 0.0;
#pragma unroll
          for (int r = 0; r < N; ++r) {
            d0 = fma(Dk.d[a * N + r], uc[r], d0);
            const double dbr = sD[b * N + r], dcr = sD[c * N + r];
            d1 = fma(dbr, su[a * N2 + r * N + c], d1);
            d2 = fma(dcr, su[a * N2 + b * N + r], d2);
          }
          const double2* ga = g + a * GROW;
          const double2 q0 = ga[0], q1 = ga[GPAIR], q2 = ga[2 * GPAIR];
          const double g00 = q0.x, g01 = q0.y, g02 = q1.x, g11 = q1.y, g12 = q2.x, g22 = q2.y;
          const double w0 = g00 * d0 + g01 * d1 + g02 * d2;
          sa[a * N2 + bc] = g01 * d0 + g11 * d1 + g12 * d2;
          sb[a * N2 + bc] = g02 * d0 + g12 * d1 + g22 * d2;
#pragma unroll
          for (int q = 0; q < N; ++q) yv[q] = fma(Dk.d[a * N + q], w0, yv[q]);
        }
      }
      __syncthreads();  // w1 / w2 complete; su is free for the next step's u
      if (active) {
#pragma unroll 1
        for (int q = 0; q < N; ++q) {
          const double dqb = sD[q * N + b], dqc = sD[q * N + c];
#pragma unroll
          for (int a = 0; a < N; ++a) {
            yv[a] = fma(dqb, sa[a * N2 + q * N + c], yv[a]);
            yv[a] = fma(dqc, sb[a * N2 + b * N + q], yv[a]);
          }
        }
      }
    } else {
      if (active) {
        // K_ii = sum_q D[q][a]^2 G00[q,b,c] + D[q][b]^2 G11[a,q,c] + D[q][c]^2 G22[a,b,q]
        //        + 2 (D[a][a] D[b][b] G01 + D[a][a] D[c][c] G02 + D[b][b] D[c][c] G12)[a,b,c]
        const double dbb = sD[b * N + b], dcc = sD[c * N + c];
#pragma unroll 1
        for (int q = 0; q < N; ++q) {
          const double g0 = su[q * N2 + bc];
          const double db = sD[q * N + b], dc = sD[q * N + c];
#pragma unroll
          for (int a = 0; a < N; ++a) {
            const double da = sD[q * N + a];
            yv[a] = fma(da * da, g0, yv[a]);
            yv[a] = fma(db * db, sa[a * N2 + q * N + c], yv[a]);
            yv[a] = fma(dc * dc, sb[a * N2 + b * N + q], yv[a]);
          }
        }
#pragma unroll
        for (int a = 0; a < N; ++a) {
          const double2* ga = g + a * GROW;
          const double daa = sD[a * N + a];
          // G01, G02, G12
          yv[a] += 2.0 * (daa * dbb * ga[0].y + daa * dcc * ga[GPAIR].x + dbb * dcc * ga[2 * GPAIR].x);
        }
      }
      __syncthreads();  // su / sa / sb are rewritten by the next element
    }
    if (ZM && wg_merge) {  // workgroup-uniform
      // the diagonal branch ends on a barrier already
      if constexpr (MODE != HEX_DIAG) __syncthreads();  // sA / sB reads done
      if (give)
#pragma unroll
        for (int a = 0; a < N; ++a) sA[(sl - 1) * N2 + a * N + b] = yv[a];
      __syncthreads();
      if (take)
#pragma unroll
        for (int a = 0; a < N; ++a) yv[a] += sA[sl * N2 + a * N + b];
      if constexpr (YM) {
        // after this thread's z-take: a column that received the z-merged
        // face passes it on (the edge node of four slots ends in one column)
        if (ygive)
#pragma unroll
          for (int a = 0; a < N; ++a) sB[(sl - GZ) * N2 + a * N + c] = yv[a];
        __syncthreads();
        if (ytake)
#pragma unroll
          for (int a = 0; a < N; ++a) yv[a] += sB[sl * N2 + a * N + c];
      }
      // the diagonal writes sA / sB (G11 / G22) at the top of the next step
      // before any barrier: every take must have read the merged faces first
      // (the action writes them only after that step's first barrier)
      if constexpr (MODE == HEX_DIAG) __syncthreads();
    }
    if (active && !give && !ygive) {
      if (k > 0) yv[0] += carry;
      const bool last = k == L - 1;
      if (!last) carry = yv[N - 1];
      const bool colslot = bcol >= 0 && ((P.cmask[pos] >> bcol) & 1ull);
      double* const cs = P.slot + ((int64_t)pos * N) * NBC + bcol;
#pragma unroll
      for (int a = 0; a < N; ++a) {
        if (a == N - 1 && !last) continue;  // carried into the next element's row 0
        const double v = yv[a];
#ifdef SEM_HEX_DIAG_NOSTORE  // diagnostic builds only: no stores
        if (!(v != v)) continue;
#endif
        if (a == 0 && k == 0 && (cf & 1)) {
          face[0] = v;
        } else if (a == N - 1 && last && (cf & 2)) {
          face[N2] = v;
        } else if (colslot) {
          cs[a * NBC] = v;
        } else {
          if constexpr (MODE == HEX_ACC)
            y[m[a]] += v;
          else
            y[m[a]] = v;
        }
      }
    }
  }
}

// Row form of the action (HEX_SET / HEX_ACC): the same
// thread / slot / chain layout, with the xi1 / xi2 transposed contractions
// done row by row.  Node row a of y needs only row a of w1 and w2, and row a
// of u is read only while row a is formed, so per row: d = D u along the
// three axes, w = G d, w1 / w2 of row a into a two-row LDS ring, barrier,
// then t_a = the xi1 / xi2 D^T contractions of row a, parked in the thread's
// own row-a entry of the u block (dead after that row's barrier); y += D[a][.]
// w0 stays in registers.  LDS per slot: u (n^3) + the ring (4 n^2) instead of
// three n^3 blocks (n = 9: 22 KB per workgroup against 53 KB), and no
// loop-invariant LDS operand can be hoisted across the row barriers.
// four waves per SIMD (<= 128 VGPRs) up to n = 9; above, the allocator
// would spill at that bound, and three waves per SIMD are what the
// three-block kernel gets there
constexpr int hex_rows_min_waves(int n) { return n <= 9 ? 4 : n <= 11 ? 3 : n <= 13 ? 2 : 1; }

template <int N, int MODE, bool TM = false>
__global__ void __launch_bounds__(hex_threads(N), hex_rows_min_waves(N))
    k_hex_rows(const double* __restrict__ u, double* __restrict__ y,
               const uint32_t* __restrict__ map, const double* __restrict__ G,
               const double* __restrict__ gD, HexLaunch P, const HexD<N> Dk) {
  static_assert(MODE == HEX_SET || MODE == HEX_ACC, "row form: the action only");
  constexpr int N2 = N * N, N3 = N2 * N, S = hex_slots(N), T = hex_threads(N), NBC = hex_nbc(N);
  constexpr int SW = S * N2;  // one plane of the ring: [slot][b*n + c]
  constexpr int GROW = 3 * N2, GPAIR = HEX_GSOA ? N2 : 1;  // factor layout (hex_g)
  __shared__ double sD[N2];
  __shared__ double sU[S * N3];
  __shared__ double sW[4 * SW];  // [row parity][w1, w2][slot][b*n + c]
  // z-merge: the xi2 = 0 face of slot s (s >= 1) handed to slot s-1
  __shared__ double sX[S > 1 ? (S - 1) * N2 : 1];
  const int tid = threadIdx.x;
  for (int i = tid; i < N2; i += T) sD[i] = gD[i];
  const int w = blockIdx.x;
  const int L = P.wg_len[w];
  const int base = P.wg_off[w];
  const int s = tid / N2;
  const int bc = tid - s * N2;
  const int b = bc / N, c = bc - b * N;
  const bool active = s < S && P.elist[base + s] >= 0;
  const int sl = active ? s : 0;
  double* const su = sU + sl * N3;
  const int bcol = hex_bcol<N>(b, c);
  const uint8_t cf = active ? P.cflag[w * S + s] : 0;
  // z-merge (planner, cflag bit 2): this slot's xi2 = 0 face is slot s-1's
  // xi2 = n-1 face at every chain step, node for node
  const bool give = (cf & 4) && c == 0;
  const bool take = active && c == N - 1 && s + 1 < S && (P.cflag[w * S + s + 1] & 4);
  bool wg_merge = false;
#pragma unroll
  for (int t = 1; t < S; ++t) wg_merge |= (P.cflag[w * S + t] & 4) != 0;
  double* const face = P.slot + P.face_base + (int64_t)(w * S + sl) * 2 * N2 + bc;
  __syncthreads();  // sD
  double carry = 0.0;
  uint32_t mn[N];
  int en = active ? P.elist[base + s] : 0;
  [[maybe_unused]] int toff[TM ? N : 1];  // template map (HexLaunch::tmpl)
  if constexpr (TM)
#pragma unroll
    for (int a = 0; a < N; ++a) toff[a] = P.tmpl[a * N2 + bc];
  if (active) {
    if constexpr (TM) {
      const uint32_t eb = P.ebase[en];
#pragma unroll
      for (int a = 0; a < N; ++a) mn[a] = eb + (uint32_t)toff[a];
    } else {
#pragma unroll
      for (int a = 0; a < N; ++a) mn[a] = map[(int64_t)en * N3 + a * N2 + bc];
    }
  }
#pragma unroll 1
  for (int k = 0; k < L; ++k) {
    const int pos = base + k * S + s;
    const int e = en;
    uint32_t m[N];
#pragma unroll
    for (int a = 0; a < N; ++a) m[a] = mn[a];
    const double2* g = hex_g<N>(G, e, bc);
    double uc[N];
    if (active) {
#pragma unroll
      for (int a = 0; a < N; ++a) uc[a] = u[m[a]];
#pragma unroll
      for (int a = 0; a < N; ++a) su[a * N2 + bc] = uc[a];
    }
    __syncthreads();  // u complete; the previous element's ring / sX reads are done
    if (active && k + 1 < L) {
      en = P.elist[pos + S];
      if constexpr (TM) {
        const uint32_t eb = P.ebase[en];
#pragma unroll
        for (int a = 0; a < N; ++a) mn[a] = eb + (uint32_t)toff[a];
      } else {
#pragma unroll
        for (int a = 0; a < N; ++a) mn[a] = map[(int64_t)en * N3 + a * N2 + bc];
      }
    }
    double yv[N];
#pragma unroll
    for (int a = 0; a < N; ++a) yv[a] = 0.0;
#pragma unroll 1
    for (int a = 0; a < N; ++a) {
      double* const w1p = sW + (a & 1) * 2 * SW + sl * N2;
      double* const w2p = w1p + SW;
      if (active) {
        double d0 = 0.0, d1 = 0.0, d2 = 0.0;
#pragma unroll
        for (int r = 0; r < N; ++r) {
          d0 = fma(Dk.d[a * N + r], uc[r], d0);
          d1 = fma(sD[b * N + r], su[a * N2 + r * N + c], d1);
          d2 = fma(sD[c * N + r], su[a * N2 + b * N + r], d2);
        }
        const double2* ga = g + a * GROW;
        const double2 q0 = ga[0], q1 = ga[GPAIR], q2 = ga[2 * GPAIR];
        const double g00 = q0.x, g01 = q0.y, g02 = q1.x, g11 = q1.y, g12 = q2.x, g22 = q2.y;
        const double w0 = g00 * d0 + g01 * d1 + g02 * d2;
        w1p[bc] = g01 * d0 + g11 * d1 + g12 * d2;
        w2p[bc] = g02 * d0 + g12 * d1 + g22 * d2;
#pragma unroll
        for (int q = 0; q < N; ++q) yv[q] = fma(Dk.d[a * N + q], w0, yv[q]);
      }
      __syncthreads();  // row a of w1 / w2 complete; row a of u is dead
      if (active) {
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < N; ++q) {
          t = fma(sD[q * N + b], w1p[q * N + c], t);
          t = fma(sD[q * N + c], w2p[b * N + q], t);
        }
        su[a * N2 + bc] = t;
      }
    }
    if (active) {
#pragma unroll
      for (int a = 0; a < N; ++a) yv[a] += su[a * N2 + bc];  // the thread's own entries
    }
    if (wg_merge) {  // workgroup-uniform
      if (active && give)
#pragma unroll
        for (int a = 0; a < N; ++a) sX[(sl - 1) * N2 + a * N + b] = yv[a];
      __syncthreads();
      if (take)
#pragma unroll
        for (int a = 0; a < N; ++a) yv[a] += sX[sl * N2 + a * N + b];
    }
    if (active && !give) {
      if (k > 0) yv[0] += carry;
      const bool last = k == L - 1;
      if (!last) carry = yv[N - 1];
      const bool colslot = bcol >= 0 && ((P.cmask[pos] >> bcol) & 1ull);
      double* const cs = P.slot + ((int64_t)pos * N) * NBC + bcol;
#pragma unroll
      for (int a = 0; a < N; ++a) {
        if (a == N - 1 && !last) continue;  // carried into the next element's row 0
        const double v = yv[a];
        if (a == 0 && k == 0 && (cf & 1)) {
          face[0] = v;
        } else if (a == N - 1 && last && (cf & 2)) {
          face[N2] = v;
        } else if (colslot) {
          cs[a * NBC] = v;
        } else {
          if constexpr (MODE == HEX_ACC)
            y[m[a]] += v;
          else
            y[m[a]] = v;
        }
      }
    }
  }
}

// y[gid[i]] (=|+=) sum of the slot values of seam node i, in plan order
template <bool ACC>
__global__ void k_hex_seam_sum(double* __restrict__ y, const uint32_t* __restrict__ gid,
                               const uint32_t* __restrict__ ptr, const uint32_t* __restrict__ idx,
                               int64_t n, const double* __restrict__ slot) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t j0 = ptr[i], j1 = ptr[i + 1];
    double v = 0.0;
    for (uint32_t j = j0; j < j1; ++j) v += slot[idx[j]];
    if (ACC)
      y[gid[i]] += v;
    else
      y[gid[i]] = v;
  }
}

// Geometry of hexahedra from equispaced element nodes (d_nodes [3][n_node]):
//   x_phys = (V^-1 (x) V^-1 (x) V^-1) X       TensorProduct.compute_coeffs_grid_eq
//                                             (sem/basis_functions.py:599-624) in 3-D
//   J[c][d] = d x_c / d xi_d                  gradient(x_phys).swapaxes(0, 1)
//                                             (sem/mapping.py:113-114)
//   det, invJ = J^-1 (cofactors)              the 3x3 twin of det_inv_2x2 (sem/linalg.py:105-115)
//   detJxW = ((det w_a) w_b) w_c              TensorQuadratureRule.xweight (sem/quadratures.py:268-275)
//   G_kl = detJxW sum_j invJ[k][j] invJ[l][j]
// The transforms act on coordinates relative to the element's node (0,0,0)
// (the constant is added back to x_phys) to keep the rounding of V^-1's
// large alternating entries off the absolute position.  Outputs may be null:
// GP: the action's pair layout (hex_g), x_phys [E][3][n^3], J / invJ
// [E][3][3][n^3], detJ / detJxW [E][n^3].  bad counts nodes with detJ <= 0.
template <int N>
__global__ void __launch_bounds__(hex_threads(N))
    k_hex_geom(const double* __restrict__ nodes, int64_t n_node, const uint32_t* __restrict__ map,
               int64_t n_elem, const double* __restrict__ gV, const double* __restrict__ gD,
               const double* __restrict__ gw, double* __restrict__ GP, double* __restrict__ xph,
               double* __restrict__ Jo, double* __restrict__ iJo, double* __restrict__ dJo,
               double* __restrict__ dJWo, unsigned long long* __restrict__ bad,
               const double* __restrict__ xrel) {
  constexpr int N2 = N * N, N3 = N2 * N, S = hex_slots(N), T = hex_threads(N);
  __shared__ double sV[N2], sD[N2], sw[N];
  __shared__ double sX[3][S * N3];
  const int tid = threadIdx.x;
  for (int i = tid; i < N2; i += T) {
    sV[i] = gV[i];
    sD[i] = gD[i];
  }
  for (int i = tid; i < N; i += T) sw[i] = gw[i];
  const int s = tid / N2;
  const int bc = tid - s * N2;
  const int b = bc / N, c = bc - b * N;
  const int sl = s < S ? s : 0;
  unsigned long long nbad = 0;
  __syncthreads();
#pragma unroll 1
  for (int64_t e0 = (int64_t)blockIdx.x * S; e0 < n_elem; e0 += (int64_t)gridDim.x * S) {
    const int64_t e = e0 + s;
    const bool active = s < S && e < n_elem;
    double x[3][N];
    double xr[3] = {0.0, 0.0, 0.0};
    double* const sx0 = sX[0] + sl * N3;
    double* const sx1 = sX[1] + sl * N3;
    double* const sx2 = sX[2] + sl * N3;
    double* const sxk[3] = {sx0, sx1, sx2};
    if (active) {
      const uint32_t g0 = map[e * N3];
#pragma unroll
      for (int k = 0; k < 3; ++k) xr[k] = nodes[k * n_node + g0];
    }
    if (xrel) {  // x_phys - x_phys(0,0,0) given (k_hex_eq2gll_pass, compensated)
      if (active)
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int a = 0; a < N; ++a) x[k][a] = xrel[(e * 3 + k) * N3 + a * N2 + bc];
    } else {  // the three passes here (uniform branch: xrel is an argument)
      if (active) {
        const uint32_t* me = map + e * N3;
        double xe[3][N];
#pragma unroll
        for (int a = 0; a < N; ++a) {
          const uint32_t gi = me[a * N2 + bc];
#pragma unroll
          for (int k = 0; k < 3; ++k) xe[k][a] = nodes[k * n_node + gi] - xr[k];
        }
        // xi0: registers
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int a = 0; a < N; ++a) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < N; ++r) v = fma(sV[a * N + r], xe[k][r], v);
            sxk[k][a * N2 + bc] = v;
          }
      }
      __syncthreads();
      if (active) {  // xi1
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int a = 0; a < N; ++a) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < N; ++r) v = fma(sV[b * N + r], sxk[k][a * N2 + r * N + c], v);
            x[k][a] = v;
          }
      }
      __syncthreads();
      if (active)
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int a = 0; a < N; ++a) sxk[k][a * N2 + bc] = x[k][a];
      __syncthreads();
      if (active) {  // xi2
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int a = 0; a < N; ++a) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < N; ++r) v = fma(sV[c * N + r], sxk[k][a * N2 + b * N + r], v);
            x[k][a] = v;  // x_phys relative to node (0,0,0)
          }
      }
    }  // xrel
    __syncthreads();
    if (active)
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int a = 0; a < N; ++a) sxk[k][a * N2 + bc] = x[k][a];
    __syncthreads();
    if (active) {
#pragma unroll
      for (int a = 0; a < N; ++a) {
        double J[3][3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          double j0 = 0.0, j1 = 0.0, j2 = 0.0;
#pragma unroll
          for (int r = 0; r < N; ++r) {
            j0 = fma(sD[a * N + r], x[k][r], j0);
            j1 = fma(sD[b * N + r], sxk[k][a * N2 + r * N + c], j1);
            j2 = fma(sD[c * N + r], sxk[k][a * N2 + b * N + r], j2);
          }
          J[k][0] = j0;
          J[k][1] = j1;
          J[k][2] = j2;
        }
        const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
        const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
        const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
        const double det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
        const double r = 1.0 / det;
        double iJ[3][3];
        iJ[0][0] = c00 * r;
        iJ[1][0] = c01 * r;
        iJ[2][0] = c02 * r;
        iJ[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * r;
        iJ[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * r;
        iJ[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * r;
        iJ[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * r;
        iJ[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * r;
        iJ[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * r;
        if (!(det > 0.0)) ++nbad;
        const double W = ((det * sw[a]) * sw[b]) * sw[c];
        const int64_t node = e * N3 + a * N2 + bc;
        if (GP) {
          double2* gp = reinterpret_cast<double2*>(GP) + hex_g_off<N>(e, bc) + a * (3 * N2);
          gp[0] = make_double2(
              W * (iJ[0][0] * iJ[0][0] + iJ[0][1] * iJ[0][1] + iJ[0][2] * iJ[0][2]),
              W * (iJ[0][0] * iJ[1][0] + iJ[0][1] * iJ[1][1] + iJ[0][2] * iJ[1][2]));
          gp[HEX_GSOA ? N2 : 1] = make_double2(
              W * (iJ[0][0] * iJ[2][0] + iJ[0][1] * iJ[2][1] + iJ[0][2] * iJ[2][2]),
              W * (iJ[1][0] * iJ[1][0] + iJ[1][1] * iJ[1][1] + iJ[1][2] * iJ[1][2]));
          gp[HEX_GSOA ? 2 * N2 : 2] = make_double2(
              W * (iJ[1][0] * iJ[2][0] + iJ[1][1] * iJ[2][1] + iJ[1][2] * iJ[2][2]),
              W * (iJ[2][0] * iJ[2][0] + iJ[2][1] * iJ[2][1] + iJ[2][2] * iJ[2][2]));
        }
        if (xph)
#pragma unroll
          for (int k = 0; k < 3; ++k) xph[(e * 3 + k) * N3 + a * N2 + bc] = x[k][a] + xr[k];
        if (Jo)
#pragma unroll
          for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int d = 0; d < 3; ++d) Jo[((e * 3 + k) * 3 + d) * N3 + a * N2 + bc] = J[k][d];
        if (iJo)
#pragma unroll
          for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int d = 0; d < 3; ++d) iJo[((e * 3 + k) * 3 + d) * N3 + a * N2 + bc] = iJ[k][d];
        if (dJo) dJo[node] = det;
        if (dJWo) dJWo[node] = W;
      }
    }
    __syncthreads();  // sX is rewritten by the next element
  }
  if (nbad) atomicAdd(bad, nbad);
}

// The equispaced -> GLL transform above p = 10 (k_hex_geom's xrel input):
// V_eq^-1 has entries up to ~170 at p = 16 (cond ~1e5) and J = D x_phys
// amplifies the rounding of plain float64 sums by ~n^2/4, so, as on
// quadrilaterals (k_geometry), every pass is a compensated dot
// product (Ogita-Rump-Oishi Dot2, semk::dot2) on coordinates relative to the
// element's node (0,0,0), the intermediate kept as hi + lo in global scratch
// (setup only).  Layout of every array: [E][3][n^3], local node a*n^2 + b*n + c.
// Pass 0: the relative element coordinates from the nodes and the map, as
// the exact difference hi + lo (two_sum): the rounding of a float64
// difference alone is amplified by cond(V_eq) (9e-11 of x_phys at p = 14).
template <int N>
__global__ void k_hex_rel_coords(const double* __restrict__ nodes, int64_t n_node,
                                 const uint32_t* __restrict__ map, int64_t n_elem,
                                 double* __restrict__ out, double* __restrict__ out_lo) {
  constexpr int N3 = N * N * N;
  const int64_t total = n_elem * 3 * N3;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ek = t / N3, e = ek / 3;
    const int node = (int)(t - ek * N3), k = (int)(ek - e * 3);
    double hi, lo;
    semk::two_sum(nodes[k * n_node + map[e * N3 + node]], -nodes[k * n_node + map[e * N3]], hi, lo);
    out[t] = hi;
    out_lo[t] = lo;
  }
}
// One pass along axis AX (0: a, 1: b, 2: c): out = V_eq^-1 (vh + vl, an
// inverse computed in extended precision) applied along AX to in = hi (+ lo),
// compensated: s_hi + s_lo ~= sum_r (vh + vl)[m][r] (in_hi + in_lo)[r] to
// about twice the working precision (Dot2 with both low parts folded in).
template <int N>
__device__ __forceinline__ void dot2x(const double* ah, const double* al, const double* bh,
                                      const double* bl, int sb, double& hi, double& lo) {
  double s = 0.0, c = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double p, ep, es;
    semk::two_prod(ah[i], bh[i * sb], p, ep);
    semk::two_sum(s, p, s, es);
    c += ep + es;
    if (bl) c = fma(ah[i], bl[i * sb], c);
    c = fma(al[i], bh[i * sb], c);
  }
  hi = s + c;
  lo = c - (hi - s);
}
template <int N, int AX>
__global__ void k_hex_eq2gll_pass(const double* __restrict__ in_hi, const double* __restrict__ in_lo,
                                  double* __restrict__ out_hi, double* __restrict__ out_lo,
                                  const double* __restrict__ vh, const double* __restrict__ vl,
                                  int64_t n_blocks) {
  constexpr int N2 = N * N, N3 = N2 * N;
  constexpr int ST = AX == 0 ? N2 : AX == 1 ? N : 1;  // stride along the axis
  __shared__ double sV[N2], sVl[N2];
  for (int i = threadIdx.x; i < N2; i += blockDim.x) {
    sV[i] = vh[i];
    sVl[i] = vl[i];
  }
  __syncthreads();
  const int64_t total = n_blocks * N3;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = t / N3;
    const int node = (int)(t - blk * N3);
    const int m = AX == 0 ? node / N2 : AX == 1 ? (node / N) % N : node % N;
    const int64_t line = blk * N3 + node - m * ST;  // the line's first node
    double hi, lo;
    dot2x<N>(&sV[m * N], &sVl[m * N], in_hi + line, in_lo ? in_lo + line : nullptr, ST, hi, lo);
    out_hi[t] = hi;
    if (out_lo) out_lo[t] = lo;
  }
}

__global__ void k_hex_zero(double* __restrict__ y, const uint32_t* __restrict__ idx, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    y[idx[t]] = 0.0;
}

// out[map[e][a][b][c]] += vals[e][a][b][c] (setup-time assembly, e.g. load vectors)
__global__ void k_hex_assemble(const uint32_t* __restrict__ e2n, const double* __restrict__ vals,
                               int64_t total, double* __restrict__ out) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x)
    unsafeAtomicAdd(out + e2n[t], vals[t]);
}

// user factors [E][6][n^3] -> the action's pair layout (hex_g)
__global__ void k_hex_pack_geom(const double* __restrict__ G, int64_t n_elem, int n,
                                double* __restrict__ GP) {
  const int64_t n2 = (int64_t)n * n, n3 = n2 * n;
  const int64_t total = n_elem * 6 * n3;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / (6 * n3);
    const int64_t rem = t - e * 6 * n3;
    const int comp = (int)(rem / n3);
    const int64_t node = rem - comp * n3;
    if (HEX_GSOA) {  // [e][a][pair][bc][2]
      const int64_t a = node / n2, bc = node - a * n2;
      GP[(((e * n + a) * 3 + comp / 2) * n2 + bc) * 2 + (comp & 1)] = G[t];
    } else {
      GP[(e * n3 + node) * 6 + comp] = G[t];
    }
  }
}

}  // namespace semh
