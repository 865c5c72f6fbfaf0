// Hexahedral (3-D) operator path of libsem_hip.so: the scatter planner (host,
// once per map), the per-order launches of sem_hex.h and the 3-D halves of
// the C ABI entry points (sem_device.hip forwards a context created with
// ndim = 3 here).  DESIGN.md §4.9 / §5.3.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <unordered_map>

#include "sem_ctx.h"
#include "sem_hex.h"

using sem::fail;
using semd::DeviceGuard;
using semd::grid_for;

struct HexState {
  int N = 0, slots = 0, threads = 0, nbc = 0;
  // launch tables (HexLaunch)
  int64_t n_wg = 0, n_pos = 0;
  int* d_wg_off = nullptr;
  int* d_wg_len = nullptr;
  int* d_elist = nullptr;
  unsigned long long* d_cmask = nullptr;
  uint8_t* d_cflag = nullptr;
  double* d_slot = nullptr;
  int64_t face_base = 0, n_slot = 0;
  // seam sums: seam node i = gid[i] sums slot[idx[ptr[i] .. ptr[i+1])]
  uint32_t* d_seam_gid = nullptr;
  uint32_t* d_seam_ptr = nullptr;
  uint32_t* d_seam_idx = nullptr;
  int64_t n_seam = 0, n_seam_writes = 0;
  uint32_t* d_zero = nullptr;  // unreferenced nodes (overwrite mode zeroes them)
  int64_t n_zero = 0;
  uint32_t* d_map = nullptr;   // the library's copy of the caller's map [E][n][n][n]
  double* d_vx = nullptr;      // V_eq^-1 hi, lo (extended-precision inverse, p >= 11)
  double* d_G = nullptr;       // stored factors, 6 per element node (pair layout, sem_hex.h hex_g)
  bool have_G = false;
  // the action's kernel: k_hex_poisson (three-block, default) or k_hex_rows
  // (row form, SEM_HEX_ROWS=1; the diagonal always runs k_hex_poisson)
  bool rows = true;
  // xi2 faces between the slots of a workgroup summed in LDS (both kernels;
  // SEM_HEX_ZMERGE=0 turns it off)
  bool zmerge = false;
  // xi1 faces between the rows of a workgroup's slot grid too (three-block
  // kernel only; SEM_HEX_YMERGE=0 turns it off)
  bool ymerge = false;
  // template map (HexLaunch::ebase / tmpl; both kernel forms): every
  // element's ids = its first node's id + one offset block (SEM_HEX_TMAP=0
  // turns it off)
  bool tmap = false;
  uint32_t* d_ebase = nullptr;
  int* d_tmpl = nullptr;
  // diagnostics (sem_plan_info)
  int64_t n_chains = 0, n_subchains = 0, chain_len = 0, n_direct = 0;

  void free_plan() {
    for (void* p : {(void*)d_wg_off, (void*)d_wg_len, (void*)d_elist, (void*)d_cmask,
                    (void*)d_cflag, (void*)d_slot, (void*)d_seam_gid, (void*)d_seam_ptr,
                    (void*)d_seam_idx, (void*)d_zero, (void*)d_ebase, (void*)d_tmpl})
      (void)hipFree(p);
    d_ebase = nullptr;
    d_tmpl = nullptr;
    tmap = false;
    d_wg_off = d_wg_len = d_elist = nullptr;
    d_cmask = nullptr;
    d_cflag = nullptr;
    d_slot = nullptr;
    d_seam_gid = d_seam_ptr = d_seam_idx = d_zero = nullptr;
    n_wg = n_pos = n_slot = n_seam = n_seam_writes = n_zero = 0;
  }
};

namespace {

#define SEM_TRY_RC(expr) \
  do {                     \
    int _rc = (expr);      \
    if (_rc) return _rc;   \
  } while (0)

int hex_check_order(int n) {
  if (n < semh::HEX_MIN_N || n > semh::HEX_MAX_N)
    return fail(SEM_E_NOTIMPL, "hexahedral kernels are built for orders 1.." +
                                   std::to_string(semh::HEX_MAX_N - 1));
  return SEM_OK;
}

template <typename T>
int upload(T** dst, const std::vector<T>& v) {
  (void)hipFree(*dst);
  *dst = nullptr;
  if (v.empty()) return SEM_OK;
  HIP_TRY(hipMalloc(dst, v.size() * sizeof(T)));
  HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return SEM_OK;
}

uint64_t face_hash(const uint32_t* f, int n2) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int j = 0; j < n2; ++j) {
    h ^= f[j] + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ull;
  }
  return h ^ (h >> 31);
}

// ---------------------------------------------------------------------------
// Planner.  Chains follow xi0: element e' succeeds e when e's face a = n-1 is
// e''s face a = 0 node for node (same (b, c) order), so one thread holds the
// shared node row of both.  Chains are cut into sub-chains of <= Lc elements
// so that the launch has enough workgroups; a workgroup runs S sub-chains of
// equal length in lockstep (slot s of step k = launch position
// wg_off + k*S + s).
//
// Every (element, node) the kernel writes is a write EVENT, except row
// a = n-1 of a non-last chain element (carried).  A node with one event is a
// plain store.  A node with several events is a SEAM node: each of its events
// goes to a slot of its own and k_hex_seam_sum adds them.  The kernel decides
// per thread and element from two small masks: a boundary column (b or c on
// the element boundary) is slotted as a whole when any of its events is on a
// seam node (cmask bit), a chain's first / last face likewise (cflag).  The
// planner replays exactly that rule, checks that every plain store hits a
// one-event node (conforming mesh) and lists the slots of each seam node.
struct HexPlanHost {
  std::vector<int> wg_off, wg_len, elist;
  std::vector<unsigned long long> cmask;
  std::vector<uint8_t> cflag;
  std::vector<uint32_t> seam_gid, seam_ptr, seam_idx, zero;
  int64_t n_slot = 0, face_base = 0, n_chains = 0, n_sub = 0, lc = 0, n_direct = 0;
};

// hash of an element face given as n^2 entries at f[i * stride1 + j * stride2]
uint64_t face_hash_strided(const uint32_t* f, int n, int stride1, int stride2) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      h ^= f[i * stride1 + j * stride2] + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
      h *= 0xBF58476D1CE4E5B9ull;
    }
  return h ^ (h >> 31);
}

int hex_build_plan(const std::vector<uint32_t>& h, int64_t E, int64_t n_node, int N,
                   int64_t resident, bool zmerge, bool ymerge, HexPlanHost& P) {
  const int N2 = N * N;
  const int64_t N3 = (int64_t)N2 * N;
  const int S = semh::hex_slots(N), NBC = semh::hex_nbc(N);
  for (size_t i = 0; i < h.size(); ++i)
    if (h[i] >= (uint64_t)n_node) return fail(SEM_E_INVALID, "element map entry >= n_node");
  // 1. successors along xi0
  std::vector<int64_t> succ(E, -1), pred(E, -1);
  {
    std::unordered_map<uint64_t, int64_t> first;
    first.reserve((size_t)E * 2);
    for (int64_t e = 0; e < E; ++e) {
      auto it = first.emplace(face_hash(&h[e * N3], N2), e);
      if (!it.second) it.first->second = -1;  // ambiguous: never chained
    }
    for (int64_t e = 0; e < E; ++e) {
      const uint32_t* fl = &h[e * N3 + (int64_t)(N - 1) * N2];
      auto it = first.find(face_hash(fl, N2));
      if (it == first.end() || it->second < 0 || it->second == e) continue;
      const int64_t e2 = it->second;
      if (std::memcmp(fl, &h[e2 * N3], sizeof(uint32_t) * N2) != 0) continue;
      if (pred[e2] >= 0) continue;
      succ[e] = e2;
      pred[e2] = e;
    }
  }
  // 2. maximal chains (heads without predecessor; then any cycle, cut anywhere)
  std::vector<int64_t> order;
  std::vector<int64_t> chain_start;
  order.reserve(E);
  {
    std::vector<uint8_t> seen(E, 0);
    auto walk = [&](int64_t e) {
      chain_start.push_back((int64_t)order.size());
      while (e >= 0 && !seen[e]) {
        seen[e] = 1;
        order.push_back(e);
        e = succ[e];
      }
    };
    for (int64_t e = 0; e < E; ++e)
      if (pred[e] < 0) walk(e);
    for (int64_t e = 0; e < E; ++e)
      if (!seen[e]) walk(e);
    chain_start.push_back((int64_t)order.size());
  }
  const int64_t n_chains = (int64_t)chain_start.size() - 1;
  // 3. sub-chains of near-equal length <= lc.  A workgroup's time grows
  //    with its sub-chain length and the launch runs in generations of
  //    `resident` workgroups, so lc minimises generations x sub-chain length
  //    (ties: the longer sub-chains, fewer seam nodes).  27^3 at p = 8: lc = 9,
  //    729 workgroups in one generation -- 0.271 against 0.278 ms per step
  //    for the round's first rule (lc = 3, 2.85 generations) and 0.275 /
  //    0.288 / 0.305 for lc = 5 / 4 / 7 (profiles/r05/hex/chain_length/).
  //    A workgroup also pays a fixed start (D into LDS, its flags, the
  //    first map rows) worth about one element step: cost = generations x
  //    (sub-chain length + 1).  Without that term the rule took sub-chains
  //    of one element at p = 1 / 3 / 6 / 7 (~1e7 DOF, many generations
  //    either way): 1.431 / 0.418 / 0.285 / 0.268 ms per step against 1.193
  //    / 0.397 / 0.277 / 0.258 with it (sub-chains of 12 / 14 / 8 / 15);
  //    the other orders keep their plan (profiles/r06/hex_chain_start/).
  //    SEM_HEX_CHAIN_START sets the term.
  int64_t lc = 1;
  {
    double start = 1.0;
    if (const char* e = std::getenv("SEM_HEX_CHAIN_START")) start = std::atof(e);
    double best = 0.0;
    for (int64_t c = 1; c <= 16; ++c) {
      int64_t nsub = 0, maxlen = 0;
      for (int64_t ch = 0; ch < n_chains; ++ch) {
        const int64_t M = chain_start[ch + 1] - chain_start[ch];
        const int64_t parts = (M + c - 1) / c;
        nsub += parts;
        maxlen = std::max(maxlen, (M + parts - 1) / parts);
      }
      const int64_t nwg = (nsub + S - 1) / S;
      const int64_t gens = resident > 0 ? (nwg + resident - 1) / resident : 1;
      const double cost = (double)gens * ((double)maxlen + start);
      if (c == 1 || cost <= best) {
        best = cost;
        lc = c;
      }
    }
  }
  if (const char* s = std::getenv("SEM_HEX_CHAIN")) lc = std::max(1, std::atoi(s));
  struct Sub {
    int64_t start, len;
  };
  std::vector<Sub> sub;
  for (int64_t ch = 0; ch < n_chains; ++ch) {
    const int64_t a0 = chain_start[ch], M = chain_start[ch + 1] - a0;
    const int64_t parts = (M + lc - 1) / lc;
    const int64_t q = M / parts, r = M % parts;
    int64_t off = a0;
    for (int64_t k = 0; k < parts; ++k) {
      const int64_t len = q + (k < r ? 1 : 0);
      sub.push_back({off, len});
      off += len;
    }
  }
  // 4. longest first, then by the smallest node id of the head element
  //    (neighbouring sub-chains share faces: on a locality-ordered node
  //    numbering they run in the same or adjacent workgroups, whatever the
  //    element order)
  std::vector<uint32_t> key(sub.size());
  for (size_t i = 0; i < sub.size(); ++i) {
    const uint32_t* me = &h[order[sub[i].start] * N3];
    key[i] = *std::min_element(me, me + N3);
  }
  {
    std::vector<size_t> idx(sub.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) {
      if (sub[x].len != sub[y].len) return sub[x].len > sub[y].len;
      return key[x] < key[y];
    });
    std::vector<Sub> sorted(sub.size());
    for (size_t i = 0; i < idx.size(); ++i) sorted[i] = sub[idx[i]];
    sub.swap(sorted);
  }
  // 5. workgroups of S equal-length sub-chains.  With the y-merge the S
  //    slots form a GY x GZ grid: row r of a workgroup is GZ sub-chains that
  //    follow each other along xi2 (xi2 = n-1 face of one = xi2 = 0 face of
  //    the next at every step), row r + 1 the xi1-neighbours of row r.  A
  //    workgroup whose first row cannot be completed (mesh edge, irregular
  //    numbering) takes the next free sub-chains of its length in order, as
  //    without the y-merge; so does the rest of a grid that ends early.
  const int GZ = semh::hex_grid_z(N), GY = S / GZ;
  const bool grid = zmerge && ymerge && GY >= 2;
  const size_t nsub = sub.size();
  // same-length neighbour along xi2 (kind 0) / xi1 (kind 1): its face 0
  // equals my face n-1 at every step
  auto face_ptr = [&](int64_t e, int kind, int side, int& st1, int& st2) -> const uint32_t* {
    // kind 0: xi2 face c = side: entries (a, b) at a*N2 + b*N; kind 1: xi1
    // face b = side: entries (a, c) at a*N2 + c
    if (kind == 0) {
      st1 = N2;
      st2 = N;
      return &h[e * N3 + side];
    }
    st1 = N2;
    st2 = 1;
    return &h[e * N3 + (int64_t)side * N];
  };
  auto same_faces = [&](int64_t i, int64_t j, int kind) -> bool {
    if (sub[i].len != sub[j].len) return false;
    for (int64_t k = 0; k < sub[i].len; ++k) {
      int a1, a2, b1, b2;
      const uint32_t* f1 = face_ptr(order[sub[i].start + k], kind, N - 1, a1, a2);
      const uint32_t* f2 = face_ptr(order[sub[j].start + k], kind, 0, b1, b2);
      for (int x = 0; x < N; ++x)
        for (int y = 0; y < N; ++y)
          if (f1[x * a1 + y * a2] != f2[x * b1 + y * b2]) return false;
    }
    return true;
  };
  std::vector<int64_t> nbr[2];
  if (grid)
    for (int kind = 0; kind < 2; ++kind) {
      nbr[kind].assign(nsub, -1);
      std::unordered_map<uint64_t, int64_t> head;
      head.reserve(nsub * 2);
      for (size_t j = 0; j < nsub; ++j) {
        int s1, s2;
        const uint32_t* f = face_ptr(order[sub[j].start], kind, 0, s1, s2);
        auto it = head.emplace(face_hash_strided(f, N, s1, s2), (int64_t)j);
        if (!it.second) it.first->second = -1;  // ambiguous
      }
      for (size_t i = 0; i < nsub; ++i) {
        int s1, s2;
        const uint32_t* f = face_ptr(order[sub[i].start], kind, N - 1, s1, s2);
        auto it = head.find(face_hash_strided(f, N, s1, s2));
        if (it == head.end() || it->second < 0 || it->second == (int64_t)i) continue;
        if (same_faces((int64_t)i, it->second, kind)) nbr[kind][i] = it->second;
      }
    }
  std::vector<int64_t> sub_wg(nsub, -1), sub_slot(nsub, -1);
  std::vector<uint8_t> grid_wg;
  int64_t pos = 0;
  size_t cur = 0;  // first sub-chain not yet placed
  std::vector<int64_t> slots(S);
  while (true) {
    while (cur < nsub && sub_wg[cur] >= 0) ++cur;
    if (cur >= nsub) break;
    const int64_t len = sub[cur].len;
    const int64_t w = (int64_t)P.wg_off.size();
    std::fill(slots.begin(), slots.end(), -1);
    int filled = 0;
    bool is_grid = false;
    if (grid) {
      int64_t rs = (int64_t)cur;
      for (int r = 0; r < GY && rs >= 0; ++r) {
        int64_t x = rs;
        int zi = 0;
        for (; zi < GZ && x >= 0; ++zi) {
          bool taken = sub_wg[x] >= 0 || sub[x].len != len;
          for (int t = 0; t < filled + zi && !taken; ++t) taken = slots[t] == x;
          if (taken) break;
          slots[filled + zi] = x;
          x = zi + 1 < GZ ? nbr[0][x] : x;
        }
        if (zi < GZ) {  // incomplete row: drop it
          for (int t = filled; t < filled + zi; ++t) slots[t] = -1;
          break;
        }
        filled += GZ;
        rs = nbr[1][slots[filled - GZ]];
      }
      is_grid = filled >= 2 * GZ;
      if (!is_grid) {
        std::fill(slots.begin(), slots.end(), -1);
        filled = 0;
      }
    }
    // the rest: the next free sub-chains of this length, in order
    for (size_t j = cur; j < nsub && filled < S && sub[j].len == len; ++j) {
      if (sub_wg[j] >= 0) continue;
      bool taken = false;
      for (int t = 0; t < filled && !taken; ++t) taken = slots[t] == (int64_t)j;
      if (!taken) slots[filled++] = (int64_t)j;
    }
    if (pos > 0x7FFFFFFFll - len * S) return fail(SEM_E_INVALID, "hex plan: too many elements");
    P.wg_off.push_back((int)pos);
    P.wg_len.push_back((int)len);
    grid_wg.push_back(is_grid ? 1 : 0);
    for (int64_t k = 0; k < len; ++k)
      for (int s = 0; s < S; ++s)
        P.elist.push_back(slots[s] >= 0 ? (int)order[sub[slots[s]].start + k] : -1);
    for (int s = 0; s < S; ++s)
      if (slots[s] >= 0) {
        sub_wg[slots[s]] = w;
        sub_slot[slots[s]] = s;
      }
    pos += len * S;
  }
  const int64_t n_wg = (int64_t)P.wg_off.size(), n_pos = pos;
  P.cmask.assign(n_pos, 0ull);
  P.cflag.assign(n_wg * S, 0);
  // 5b. z-merge: slot s of a workgroup hands its xi2 = 0 face to slot s-1
  //     when, at every chain step, that face IS slot s-1's xi2 = n-1 face
  //     node for node (same (a, b)); the kernel sums it in LDS.  In a grid
  //     workgroup only within a row.  y-merge: slot s hands its xi1 = 0 face
  //     to slot s - GZ likewise (same (a, c)).
  std::vector<uint8_t> zm(n_wg * S, 0), ym(n_wg * S, 0);
  auto elem_at = [&](int64_t w, int64_t k, int s) { return P.elist[P.wg_off[w] + k * S + s]; };
  if (zmerge)
    for (int64_t w = 0; w < n_wg; ++w)
      for (int s = 1; s < S; ++s) {
        if (grid_wg[w] && s % GZ == 0) continue;
        bool ok = true;
        for (int64_t k = 0; k < P.wg_len[w] && ok; ++k) {
          const int e1 = elem_at(w, k, s - 1), e2 = elem_at(w, k, s);
          if (e1 < 0 || e2 < 0) {
            ok = false;
            break;
          }
          const uint32_t* m1 = &h[(int64_t)e1 * N3];
          const uint32_t* m2 = &h[(int64_t)e2 * N3];
          for (int ab = 0; ab < N2 && ok; ++ab) ok = m1[ab * N + N - 1] == m2[ab * N];
        }
        zm[w * S + s] = ok ? 1 : 0;
      }
  if (grid)
    for (int64_t w = 0; w < n_wg; ++w) {
      if (!grid_wg[w]) continue;
      for (int s = GZ; s < S; ++s) {
        bool ok = true;
        for (int64_t k = 0; k < P.wg_len[w] && ok; ++k) {
          const int e1 = elem_at(w, k, s - GZ), e2 = elem_at(w, k, s);
          if (e1 < 0 || e2 < 0) {
            ok = false;
            break;
          }
          const uint32_t* m1 = &h[(int64_t)e1 * N3];
          const uint32_t* m2 = &h[(int64_t)e2 * N3];
          for (int a = 0; a < N && ok; ++a)
            for (int c = 0; c < N && ok; ++c) ok = m1[a * N2 + (N - 1) * N + c] == m2[a * N2 + c];
        }
        ym[w * S + s] = ok ? 1 : 0;
      }
    }
  // a thread whose column is handed over emits no write of its own (the
  // kernel's give / ygive, sem_hex.h)
  auto merged = [&](int64_t w, int64_t s, int b, int c) {
    if (c == 0 && zm[w * S + s]) return true;
    return b == 0 && ym[w * S + s] && !(c == 0 && zm[w * S + s - GZ]);
  };
  // 6. events per node
  std::vector<uint8_t> cnt(n_node, 0);
  auto bump = [&](uint32_t g) {
    if (cnt[g] < 255) ++cnt[g];
  };
  for (size_t i = 0; i < sub.size(); ++i) {
    const int64_t len = sub[i].len;
    for (int64_t k = 0; k < len; ++k) {
      const uint32_t* me = &h[order[sub[i].start + k] * N3];
      const int amax = (k == len - 1) ? N : N - 1;
      for (int64_t t = 0; t < (int64_t)amax * N2; ++t)
        if (!merged(sub_wg[i], sub_slot[i], (int)((t / N) % N), (int)(t % N))) bump(me[t]);
    }
  }
  // 7. face flags, column masks
  auto bcol_of = [&](int b, int c) -> int {
    if (b == 0) return c;
    if (b == N - 1) return 3 * N - 4 + c;
    if (c == 0) return N + 2 * (b - 1);
    if (c == N - 1) return N + 2 * (b - 1) + 1;
    return -1;
  };
  for (size_t i = 0; i < sub.size(); ++i) {
    const int64_t len = sub[i].len;
    const uint32_t* hd = &h[order[sub[i].start] * N3];
    const uint32_t* tl = &h[order[sub[i].start + len - 1] * N3 + (int64_t)(N - 1) * N2];
    uint8_t f = 0;
    for (int j = 0; j < N2; ++j) {
      if (cnt[hd[j]] > 1) f |= 1;
      if (cnt[tl[j]] > 1) f |= 2;
    }
    if (zm[sub_wg[i] * S + sub_slot[i]]) f |= 4;
    if (ym[sub_wg[i] * S + sub_slot[i]]) f |= 8;
    P.cflag[sub_wg[i] * S + sub_slot[i]] = f;
    for (int64_t k = 0; k < len; ++k) {
      const int64_t p = P.wg_off[sub_wg[i]] + k * S + sub_slot[i];
      const uint32_t* me = &h[order[sub[i].start + k] * N3];
      unsigned long long mask = 0;
      for (int b = 0; b < N; ++b)
        for (int c = 0; c < N; ++c) {
          const int bcol = bcol_of(b, c);
          if (bcol < 0 || merged(sub_wg[i], sub_slot[i], b, c)) continue;
          for (int a = 0; a < N; ++a) {
            if (a == N - 1 && k < len - 1) continue;
            if (a == 0 && k == 0 && (f & 1)) continue;
            if (a == N - 1 && k == len - 1 && (f & 2)) continue;
            if (cnt[me[a * N2 + b * N + c]] > 1) {
              mask |= 1ull << bcol;
              break;
            }
          }
        }
      P.cmask[p] = mask;
    }
  }
  // 8. replay the kernel's rule: plain stores must hit one-event nodes; the
  //    slotted events of each seam node, in a fixed order (counting sort)
  P.face_base = n_pos * N * NBC;
  P.n_slot = P.face_base + n_wg * S * 2 * N2;
  if (P.n_slot >= 0xFFFFFFFFll) return fail(SEM_E_INVALID, "hex plan: slot space exceeds 2^32");
  std::vector<uint32_t> scount(n_node + 1, 0);
  int64_t n_direct = 0;
  auto for_events = [&](auto&& fn) -> int {
    for (size_t i = 0; i < sub.size(); ++i) {
      const int64_t len = sub[i].len, w = sub_wg[i], s = sub_slot[i];
      const uint8_t f = P.cflag[w * S + s];
      for (int64_t k = 0; k < len; ++k) {
        const int64_t p = P.wg_off[w] + k * S + s;
        const uint32_t* me = &h[order[sub[i].start + k] * N3];
        const unsigned long long mask = P.cmask[p];
        for (int b = 0; b < N; ++b)
          for (int c = 0; c < N; ++c) {
            const int bc = b * N + c, bcol = bcol_of(b, c);
            if (merged(w, s, b, c)) continue;
            const bool colslot = bcol >= 0 && ((mask >> bcol) & 1ull);
            for (int a = 0; a < N; ++a) {
              if (a == N - 1 && k < len - 1) continue;
              const uint32_t g = me[a * N2 + bc];
              int64_t sidx = -1;
              if (a == 0 && k == 0 && (f & 1))
                sidx = P.face_base + (w * S + s) * 2 * N2 + bc;
              else if (a == N - 1 && k == len - 1 && (f & 2))
                sidx = P.face_base + (w * S + s) * 2 * N2 + N2 + bc;
              else if (colslot)
                sidx = (p * N + a) * NBC + bcol;
              if (int rc = fn(g, sidx, (int64_t)i)) return rc;
            }
          }
      }
    }
    return SEM_OK;
  };
  int rc = for_events([&](uint32_t g, int64_t sidx, int64_t) -> int {
    if (sidx < 0) {
      if (cnt[g] != 1)
        return fail(SEM_E_NOTIMPL,
                    "hex plan: a node inside an element column is shared (non-conforming mesh)");
      ++n_direct;
    } else {
      ++scount[g];
    }
    return SEM_OK;
  });
  if (rc) return rc;
  std::vector<uint32_t> start(n_node + 1, 0);
  for (int64_t g = 0; g < n_node; ++g) start[g + 1] = start[g] + scount[g];
  const uint32_t n_writes = start[n_node];
  P.seam_idx.assign(n_writes, 0);
  std::vector<uint32_t> fill(start.begin(), start.end() - 1);
  for_events([&](uint32_t g, int64_t sidx, int64_t) -> int {
    if (sidx >= 0) P.seam_idx[fill[g]++] = (uint32_t)sidx;
    return SEM_OK;
  });
  P.seam_ptr.push_back(0);
  for (int64_t g = 0; g < n_node; ++g) {
    if (scount[g]) {
      P.seam_gid.push_back((uint32_t)g);
      P.seam_ptr.push_back(start[g + 1]);
    }
    if (cnt[g] == 0) P.zero.push_back((uint32_t)g);
  }
  P.n_chains = n_chains;
  P.n_sub = (int64_t)sub.size();
  P.lc = lc;
  P.n_direct = n_direct;
  return SEM_OK;
}

// ---------------------------------------------------------------------------
template <int N>
int launch_hex_apply(sem_ctx* c, int mode, const double* u, double* y, hipStream_t st) {
  HexState* H = c->hex;
  const semh::HexLaunch L{H->d_wg_off, H->d_wg_len, H->d_elist,   H->d_cmask,
                          H->d_cflag,  H->d_slot,   H->face_base, H->d_ebase, H->d_tmpl};
  const dim3 g((unsigned)H->n_wg), b(semh::hex_threads(N));
  semh::HexD<N> Dk;
  for (int i = 0; i < N * N; ++i) Dk.d[i] = c->hD[i];
  if (H->rows && H->tmap && mode == semh::HEX_SET)
    hipLaunchKernelGGL((semh::k_hex_rows<N, semh::HEX_SET, true>), g, b, 0, st, u, y, H->d_map,
                       H->d_G, c->d_D, L, Dk);
  else if (H->rows && H->tmap && mode == semh::HEX_ACC)
    hipLaunchKernelGGL((semh::k_hex_rows<N, semh::HEX_ACC, true>), g, b, 0, st, u, y, H->d_map,
                       H->d_G, c->d_D, L, Dk);
  else if (H->rows && mode == semh::HEX_SET)
    hipLaunchKernelGGL((semh::k_hex_rows<N, semh::HEX_SET>), g, b, 0, st, u, y, H->d_map, H->d_G,
                       c->d_D, L, Dk);
  else if (H->rows && mode == semh::HEX_ACC)
    hipLaunchKernelGGL((semh::k_hex_rows<N, semh::HEX_ACC>), g, b, 0, st, u, y, H->d_map, H->d_G,
                       c->d_D, L, Dk);
  else if (H->tmap && mode == semh::HEX_SET)
    hipLaunchKernelGGL((semh::k_hex_poisson<N, semh::HEX_SET, true>), g, b, 0, st, u, y,
                       H->d_map, H->d_G, c->d_D, L, Dk);
  else if (H->tmap && mode == semh::HEX_ACC)
    hipLaunchKernelGGL((semh::k_hex_poisson<N, semh::HEX_ACC, true>), g, b, 0, st, u, y,
                       H->d_map, H->d_G, c->d_D, L, Dk);
  else if (H->tmap)
    hipLaunchKernelGGL((semh::k_hex_poisson<N, semh::HEX_DIAG, true>), g, b, 0, st, u, y,
                       H->d_map, H->d_G, c->d_D, L, Dk);
  else if (mode == semh::HEX_SET)
    hipLaunchKernelGGL((semh::k_hex_poisson<N, semh::HEX_SET>), g, b, 0, st, u, y, H->d_map,
                       H->d_G, c->d_D, L, Dk);
  else if (mode == semh::HEX_ACC)
    hipLaunchKernelGGL((semh::k_hex_poisson<N, semh::HEX_ACC>), g, b, 0, st, u, y, H->d_map,
                       H->d_G, c->d_D, L, Dk);
  else
    hipLaunchKernelGGL((semh::k_hex_poisson<N, semh::HEX_DIAG>), g, b, 0, st, u, y, H->d_map,
                       H->d_G, c->d_D, L, Dk);
  HIP_TRY(hipGetLastError());
  if (H->n_seam) {
    const dim3 gs(grid_for(H->n_seam, 256, 8192)), bs(256);
    if (mode == semh::HEX_ACC)
      hipLaunchKernelGGL(semh::k_hex_seam_sum<true>, gs, bs, 0, st, y, H->d_seam_gid,
                         H->d_seam_ptr, H->d_seam_idx, H->n_seam, H->d_slot);
    else
      hipLaunchKernelGGL(semh::k_hex_seam_sum<false>, gs, bs, 0, st, y, H->d_seam_gid,
                         H->d_seam_ptr, H->d_seam_idx, H->n_seam, H->d_slot);
    HIP_TRY(hipGetLastError());
  }
  return SEM_OK;
}

// from this many nodes per line (p >= 11) the equispaced -> GLL transform
// runs as three compensated passes (k_hex_eq2gll_pass) before k_hex_geom:
// float64 sums lose 7e-12 (p = 12) to 1e-8 (p = 16) of the action against
// the extended-precision oracle (oracle
// hex_poisson_apply_extended); at p <= 10 the plain passes stay (4.7e-13)
constexpr int HEX_DOT2_MIN_N = 12;

// V_eq^-1 as hi + lo doubles, from V_eq built and inverted in x87 extended
// precision on the GLL nodes of the context's basis: the float64 inverse the
// caller passes is itself off by ~cond(V_eq) eps (1e-11 at p = 16), which the
// compensated passes would otherwise carry into x_phys.  Only for the standard
// GLL basis (the baked table reproduces the context's D bit for bit);
// otherwise hi = the caller's inverse, lo = 0.
int eq2gll_hilo(sem_ctx* c, double* hi, double* lo) {
  const int n = c->n;
  std::vector<double> xn(n), bw(n), qw(n), D((size_t)n * n);
  bool gll = sem::gll_table(c->p, xn.data(), bw.data(), qw.data()) == SEM_OK;
  if (gll) {
    sem::diff_matrix(n, xn.data(), bw.data(), D.data());
    gll = std::memcmp(D.data(), c->hD, sizeof(double) * n * n) == 0;
  }
  if (!gll) {
    HIP_TRY(hipMemcpy(hi, c->d_Vinv, sizeof(double) * n * n, hipMemcpyDeviceToHost));
    for (int i = 0; i < n * n; ++i) lo[i] = 0.0;
    return SEM_OK;
  }
  std::vector<long double> a((size_t)n * 2 * n, 0.0L);
  for (int i = 0; i < n; ++i) {
    const long double x = -1.0L + 2.0L * i / (long double)(n - 1);
    int hit = -1;
    long double sum = 0.0L;
    for (int j = 0; j < n && hit < 0; ++j) {
      const long double d = x - (long double)xn[j];
      if (d == 0.0L) hit = j;
      else sum += (long double)bw[j] / d;
    }
    for (int j = 0; j < n; ++j)
      a[(size_t)i * 2 * n + j] =
          hit >= 0 ? (j == hit ? 1.0L : 0.0L) : ((long double)bw[j] / (x - (long double)xn[j])) / sum;
    a[(size_t)i * 2 * n + n + i] = 1.0L;
  }
  for (int col = 0; col < n; ++col) {  // Gauss-Jordan, partial pivoting
    int piv = col;
    for (int r = col + 1; r < n; ++r)
      if (fabsl(a[(size_t)r * 2 * n + col]) > fabsl(a[(size_t)piv * 2 * n + col])) piv = r;
    if (piv != col)
      for (int j = 0; j < 2 * n; ++j) std::swap(a[(size_t)col * 2 * n + j], a[(size_t)piv * 2 * n + j]);
    const long double dg = a[(size_t)col * 2 * n + col];
    for (int j = 0; j < 2 * n; ++j) a[(size_t)col * 2 * n + j] /= dg;
    for (int r = 0; r < n; ++r) {
      if (r == col) continue;
      const long double f = a[(size_t)r * 2 * n + col];
      for (int j = 0; j < 2 * n; ++j) a[(size_t)r * 2 * n + j] -= f * a[(size_t)col * 2 * n + j];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      const long double v = a[(size_t)i * 2 * n + n + j];
      hi[i * n + j] = (double)v;
      lo[i * n + j] = (double)(v - (long double)hi[i * n + j]);
    }
  return SEM_OK;
}

template <int N>
int launch_hex_geom(sem_ctx* c, const double* nodes, double* GP, double* xph, double* J,
                    double* iJ, double* dJ, double* dJW, hipStream_t st) {
  HexState* H = c->hex;
  constexpr int S = semh::hex_slots(N), N3 = N * N * N;
  const int64_t nb = std::min<int64_t>((c->n_elem + S - 1) / S, 16384);
  double* buf[4] = {nullptr, nullptr, nullptr, nullptr};
  const double* xrel = nullptr;
  if constexpr (N >= HEX_DOT2_MIN_N) {
    // relative coordinates (R, Rl), then -> (A, Al) -> (R, Rl) -> A along xi0, xi1, xi2
    const int64_t total = c->n_elem * 3 * N3;
    if (!H->d_vx) HIP_TRY(hipMalloc(&H->d_vx, 2 * N * N * sizeof(double)));
    {
      std::vector<double> vx(2 * N * N);
      SEM_TRY_RC(eq2gll_hilo(c, vx.data(), vx.data() + N * N));
      HIP_TRY(hipMemcpy(H->d_vx, vx.data(), vx.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    for (double*& b : buf) HIP_TRY(hipMallocAsync((void**)&b, total * sizeof(double), st));
    const dim3 g(grid_for(total, 256, 16384)), bl(256);
    const double *vh = H->d_vx, *vl = H->d_vx + N * N;
    hipLaunchKernelGGL(semh::k_hex_rel_coords<N>, g, bl, 0, st, nodes, c->n_node, H->d_map,
                       c->n_elem, buf[0], buf[3]);
    hipLaunchKernelGGL((semh::k_hex_eq2gll_pass<N, 0>), g, bl, 0, st, buf[0], buf[3], buf[1],
                       buf[2], vh, vl, c->n_elem * 3);
    hipLaunchKernelGGL((semh::k_hex_eq2gll_pass<N, 1>), g, bl, 0, st, buf[1], buf[2], buf[0],
                       buf[3], vh, vl, c->n_elem * 3);
    hipLaunchKernelGGL((semh::k_hex_eq2gll_pass<N, 2>), g, bl, 0, st, buf[0], buf[3], buf[1],
                       nullptr, vh, vl, c->n_elem * 3);
    HIP_TRY(hipGetLastError());
    xrel = buf[1];
  }
  hipLaunchKernelGGL(semh::k_hex_geom<N>, dim3((unsigned)nb), dim3(semh::hex_threads(N)), 0, st,
                     nodes, c->n_node, H->d_map, c->n_elem, c->d_Vinv, c->d_D, c->d_w, GP, xph, J,
                     iJ, dJ, dJW, c->d_bad, xrel);
  HIP_TRY(hipGetLastError());
  for (double* b : buf)
    if (b) HIP_TRY(hipFreeAsync(b, st));
  return SEM_OK;
}

#define HEX_DISPATCH(rc, n, FN, ...)            \
  switch (n) {                                  \
    case 2: rc = FN<2>(__VA_ARGS__); break;     \
    case 3: rc = FN<3>(__VA_ARGS__); break;     \
    case 4: rc = FN<4>(__VA_ARGS__); break;     \
    case 5: rc = FN<5>(__VA_ARGS__); break;     \
    case 6: rc = FN<6>(__VA_ARGS__); break;     \
    case 7: rc = FN<7>(__VA_ARGS__); break;     \
    case 8: rc = FN<8>(__VA_ARGS__); break;     \
    case 9: rc = FN<9>(__VA_ARGS__); break;     \
    case 10: rc = FN<10>(__VA_ARGS__); break;   \
    case 11: rc = FN<11>(__VA_ARGS__); break;   \
    case 12: rc = FN<12>(__VA_ARGS__); break;   \
    case 13: rc = FN<13>(__VA_ARGS__); break;   \
    case 14: rc = FN<14>(__VA_ARGS__); break;   \
    case 15: rc = FN<15>(__VA_ARGS__); break;   \
    case 16: rc = FN<16>(__VA_ARGS__); break;   \
    case 17: rc = FN<17>(__VA_ARGS__); break;   \
    default: rc = fail(SEM_E_NOTIMPL, "hexahedral order out of range"); break; \
  }
static_assert(semh::HEX_MAX_N == 17, "HEX_DISPATCH lists n = 2..17");

// workgroups of the element kernel resident per CU (LDS and VGPR bound)
template <int N>
int hex_wgs_per_cu(bool rows, int* out) {
  int nb = 0;
  const void* k = rows ? reinterpret_cast<const void*>(&semh::k_hex_rows<N, semh::HEX_SET>)
                       : reinterpret_cast<const void*>(&semh::k_hex_poisson<N, semh::HEX_SET>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, semh::hex_threads(N), 0) !=
      hipSuccess) {
    (void)hipGetLastError();
    nb = 0;
  }
  *out = nb;
  return SEM_OK;
}

int need_map(const sem_ctx* c) {
  if (!c->have_basis) return fail(SEM_E_STATE, "sem_set_basis must precede this call");
  if (!c->hex->d_map) return fail(SEM_E_STATE, "sem_set_map must precede this call");
  return SEM_OK;
}

}  // namespace

namespace semh {

// the row form by default where the three-block kernel's LDS
// (3 S n^3 doubles) exceeds 64 KiB: n >= 14
static bool hex_rows_default(int n) {
  const int64_t lds = 8 * (3 * (int64_t)hex_slots(n) * n * n * n + (int64_t)n * n);
  return lds > 65536;
}

int ctx_init(sem_ctx* c) {
  int rc = hex_check_order(c->n);
  if (rc) return rc;
  if (c->dpn != 1) return fail(SEM_E_NOTIMPL, "hexahedral operators: dofs_per_node == 1 only");
  c->hex = new HexState();
  c->hex->N = c->n;
  c->hex->slots = hex_slots(c->n);
  c->hex->threads = hex_threads(c->n);
  c->hex->nbc = hex_nbc(c->n);
  // the row form only on request (SEM_HEX_ROWS=1): with the z-merge in both
  // kernels the three-block kernel is as fast or faster at every order
  // measured (p = 2 / 4 / 6, DESIGN.md §4.9, profiles/r05/hex/zmerge_w1/)
  // and above p = 12, where the three-block kernel's 3 n^3 doubles of LDS
  // would leave one workgroup (of one element slot) per CU
  const char* re = std::getenv("SEM_HEX_ROWS");
  c->hex->rows = re ? std::atoi(re) != 0 : hex_rows_default(c->n);
  const char* ze = std::getenv("SEM_HEX_ZMERGE");
  c->hex->zmerge = HEX_ZMERGE && !(ze && std::atoi(ze) == 0);
  // y-merge by default at n <= 4 (p <= 3), where it measured faster (p = 1 /
  // 2 / 3: 1.530 -> 1.429, 0.589 -> 0.544, 0.430 -> 0.415 ms per step at
  // ~1e7 DOF); at p = 4 / 7 its extra barrier per step outweighs the seams
  // it removes (0.324 -> 0.328, 0.266 -> 0.275; profiles/r06/hex_ymerge/).
  // SEM_HEX_YMERGE=1 / 0 forces it on / off.
  const char* ye = std::getenv("SEM_HEX_YMERGE");
  const bool ywant = ye ? std::atoi(ye) != 0 : c->n <= 4;
  c->hex->ymerge = ywant && c->hex->zmerge && !c->hex->rows && hex_grid_z(c->n) < hex_slots(c->n);
  return SEM_OK;
}

void ctx_free(sem_ctx* c) {
  if (!c->hex) return;
  c->hex->free_plan();
  (void)hipFree(c->hex->d_map);
  (void)hipFree(c->hex->d_G);
  (void)hipFree(c->hex->d_vx);
  delete c->hex;
  c->hex = nullptr;
}

int set_map(sem_ctx* c, const uint32_t* d_e2n, hipStream_t st) {
  HexState* H = c->hex;
  const int N = c->n;
  const int64_t N3 = (int64_t)N * N * N;
  const size_t count = (size_t)c->n_elem * N3;
  std::vector<uint32_t> h(count);
  HIP_TRY(hipMemcpyAsync(h.data(), d_e2n, count * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (!c->n_cu) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) ==
            hipSuccess &&
        ncu > 0)
      c->n_cu = ncu;
  }
  int wpc = 0, rc = SEM_OK;
  HEX_DISPATCH(rc, N, hex_wgs_per_cu, H->rows, &wpc);
  if (rc) return rc;
  const int64_t resident = (int64_t)std::max(c->n_cu, 1) * std::max(wpc, 1);
  HexPlanHost P;
  rc = hex_build_plan(h, c->n_elem, c->n_node, N, resident, H->zmerge, H->ymerge, P);
  if (rc) return rc;
  c->epoch++;
  c->map_epoch++;
  H->free_plan();
  (void)hipFree(H->d_map);
  H->d_map = nullptr;
  HIP_TRY(hipMalloc(&H->d_map, count * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(H->d_map, h.data(), count * sizeof(uint32_t), hipMemcpyHostToDevice));
  if ((rc = upload(&H->d_wg_off, P.wg_off)) || (rc = upload(&H->d_wg_len, P.wg_len)) ||
      (rc = upload(&H->d_elist, P.elist)) || (rc = upload(&H->d_cmask, P.cmask)) ||
      (rc = upload(&H->d_cflag, P.cflag)) || (rc = upload(&H->d_seam_gid, P.seam_gid)) ||
      (rc = upload(&H->d_seam_ptr, P.seam_ptr)) || (rc = upload(&H->d_seam_idx, P.seam_idx)) ||
      (rc = upload(&H->d_zero, P.zero)))
    return rc;
  // template map: one offset block shared by every element (structured
  // numberings); both kernel forms and the diagonal
  {
    const char* te = std::getenv("SEM_HEX_TMAP");
    bool ok = c->n_elem > 0 && !(te && std::atoi(te) == 0);
    std::vector<int> tmpl((size_t)N3);
    std::vector<uint32_t> eb;
    if (ok) {
      for (int64_t i = 0; i < N3 && ok; ++i) {
        const int64_t d = (int64_t)h[i] - (int64_t)h[0];
        ok = d >= INT32_MIN && d <= INT32_MAX;
        tmpl[(size_t)i] = (int)d;
      }
      eb.resize((size_t)c->n_elem);
      for (int64_t e = 0; e < c->n_elem && ok; ++e) {
        const uint32_t* me = &h[(size_t)e * N3];
        eb[(size_t)e] = me[0];
        for (int64_t i = 1; i < N3 && ok; ++i) ok = me[i] == me[0] + (uint32_t)tmpl[(size_t)i];
      }
    }
    if (ok) {
      if ((rc = upload(&H->d_ebase, eb)) || (rc = upload(&H->d_tmpl, tmpl))) return rc;
      H->tmap = true;
    }
  }
  H->n_wg = (int64_t)P.wg_off.size();
  H->n_pos = (int64_t)P.elist.size();
  H->face_base = P.face_base;
  H->n_slot = P.n_slot;
  H->n_seam = (int64_t)P.seam_gid.size();
  H->n_seam_writes = (int64_t)P.seam_idx.size();
  H->n_zero = (int64_t)P.zero.size();
  H->n_chains = P.n_chains;
  H->n_subchains = P.n_sub;
  H->chain_len = P.lc;
  H->n_direct = P.n_direct;
  if (H->n_seam) HIP_TRY(hipMalloc(&H->d_slot, std::max<int64_t>(H->n_slot, 1) * sizeof(double)));
  // geometry belonged to the previous map
  (void)hipFree(H->d_G);
  H->d_G = nullptr;
  H->have_G = false;
  c->d_e2n = d_e2n;
  return SEM_OK;
}

static int ensure_G(sem_ctx* c) {
  HexState* H = c->hex;
  if (!H->d_G) {
    const size_t bytes = (size_t)c->n_elem * 6 * c->n * c->n * c->n * sizeof(double);
    HIP_TRY(hipMalloc(&H->d_G, bytes));
  }
  return SEM_OK;
}

int geom_from_nodes(sem_ctx* c, const double* d_nodes, int op_kind, int64_t* n_bad,
                    hipStream_t st) {
  if (op_kind != SEM_OP_POISSON)
    return fail(SEM_E_NOTIMPL, "hexahedral operators: Poisson only");
  int rc = need_map(c);
  if (rc) return rc;
  if ((rc = ensure_G(c))) return rc;
  c->epoch++;
  HIP_TRY(hipMemsetAsync(c->d_bad, 0, sizeof(unsigned long long), st));
  HEX_DISPATCH(rc, c->n, launch_hex_geom, c, d_nodes, c->hex->d_G, nullptr, nullptr, nullptr,
               nullptr, nullptr, st);
  if (rc) return rc;
  unsigned long long bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, c->d_bad, sizeof(bad), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (n_bad) *n_bad = (int64_t)bad;
  if (bad) {
    c->hex->have_G = false;
    return fail(SEM_E_DETJ, "detJ <= 0 at " + std::to_string(bad) + " quadrature nodes");
  }
  c->hex->have_G = true;
  return SEM_OK;
}

int geom_fields(sem_ctx* c, const double* d_nodes, double* x_phys, double* J, double* invJ,
                double* detJ, double* detJxW, hipStream_t st) {
  int rc = need_map(c);
  if (rc) return rc;
  HIP_TRY(hipMemsetAsync(c->d_bad, 0, sizeof(unsigned long long), st));
  HEX_DISPATCH(rc, c->n, launch_hex_geom, c, d_nodes, nullptr, x_phys, J, invJ, detJ, detJxW,
               st);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(st));
  return SEM_OK;
}

int set_geom(sem_ctx* c, const double* d_G, int op_kind, hipStream_t st) {
  if (op_kind != SEM_OP_POISSON)
    return fail(SEM_E_NOTIMPL, "hexahedral operators: Poisson only");
  int rc = need_map(c);
  if (rc) return rc;
  if ((rc = ensure_G(c))) return rc;
  c->epoch++;
  const int64_t total = c->n_elem * 6 * c->n * c->n * c->n;
  hipLaunchKernelGGL(k_hex_pack_geom, dim3(grid_for(total)), dim3(256), 0, st, d_G, c->n_elem,
                     c->n, c->hex->d_G);
  HIP_TRY(hipGetLastError());
  c->hex->have_G = true;
  return SEM_OK;
}

int apply(sem_ctx* c, int op_kind, const double* u, double* y, int flags, hipStream_t st) {
  if (op_kind != SEM_OP_POISSON)
    return fail(SEM_E_NOTIMPL, "hexahedral operators: Poisson only");
  if (flags & ~(SEM_APPLY_ACCUMULATE | SEM_APPLY_SKIP_ZERO))
    return fail(SEM_E_INVALID, "sem_apply flags not supported on hexahedra");
  int rc = need_map(c);
  if (rc) return rc;
  HexState* H = c->hex;
  if (!H->have_G) return fail(SEM_E_STATE, "geometry for this operator has not been computed");
  const bool acc = flags & SEM_APPLY_ACCUMULATE;
  if (!acc && !(flags & SEM_APPLY_SKIP_ZERO) && H->n_zero)
    if ((rc = zero_shared(c, y, st))) return rc;
  HEX_DISPATCH(rc, c->n, launch_hex_apply, c, acc ? HEX_ACC : HEX_SET, u, y, st);
  return rc;
}

int diag(sem_ctx* c, int op_kind, double* d, hipStream_t st) {
  if (op_kind != SEM_OP_POISSON) return fail(SEM_E_NOTIMPL, "sem_diag: Poisson only");
  int rc = need_map(c);
  if (rc) return rc;
  if (!c->hex->have_G) return fail(SEM_E_STATE, "geometry/map not set");
  if (c->hex->n_zero && (rc = zero_shared(c, d, st))) return rc;
  HEX_DISPATCH(rc, c->n, launch_hex_apply, c, HEX_DIAG, nullptr, d, st);
  return rc;
}

int zero_shared(sem_ctx* c, double* y, hipStream_t st) {
  HexState* H = c->hex;
  if (!H->d_map) return fail(SEM_E_STATE, "map must be set");
  if (H->n_zero) {
    hipLaunchKernelGGL(semh::k_hex_zero, dim3(grid_for(H->n_zero, 256, 4096)), dim3(256), 0, st, y,
                       H->d_zero, H->n_zero);
    HIP_TRY(hipGetLastError());
  }
  return SEM_OK;
}

int plan_info(const sem_ctx* c, int64_t* info, int n_info) {
  const HexState* H = c->hex;
  // [0] workgroups, [1] zero list, [2] atomic groups (0), [3] conforming (1),
  // [4] element slots per workgroup, [5] chains (maximal), [6] sub-chain
  // length cap, [7] launch positions, [8] sub-chains, [9] seam nodes,
  // [10] slotted writes, [11] plain stores, [12] threads per workgroup,
  // [13] ndim (3), [14] geometry ready, [15] action kernel (1 row form,
  // 0 three-block), [16] z-merge in the plan, [17] y-merge: slots per grid
  // row (0: off), [18] template map
  const int64_t v[] = {H->n_wg,        H->n_zero, 0,
                       1,              H->slots,  H->n_chains,
                       H->chain_len,   H->n_pos,  H->n_subchains,
                       H->n_seam,      H->n_seam_writes, H->n_direct,
                       H->threads,     3,         H->have_G ? 1 : 0,
                       H->rows ? 1 : 0, H->zmerge ? 1 : 0, H->ymerge ? hex_grid_z(H->N) : 0,
                       H->tmap ? 1 : 0};
  const int nv = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n_info; ++i) info[i] = i < nv ? v[i] : 0;
  return SEM_OK;
}

int zero_list(const sem_ctx* c, std::vector<uint32_t>* nodes, bool* only_unreferenced) {
  const HexState* H = c->hex;
  nodes->assign((size_t)H->n_zero, 0u);
  *only_unreferenced = true;
  if (H->n_zero)
    HIP_TRY(hipMemcpy(nodes->data(), H->d_zero, H->n_zero * sizeof(uint32_t),
                      hipMemcpyDeviceToHost));
  return SEM_OK;
}

int assemble(sem_ctx* c, const double* vals, double* out, int accumulate, hipStream_t st) {
  HexState* H = c->hex;
  if (!H->d_map) return fail(SEM_E_STATE, "sem_set_map must precede sem_assemble");
  if (!accumulate) HIP_TRY(hipMemsetAsync(out, 0, c->n_node * sizeof(double), st));
  const int64_t total = c->n_elem * c->n * c->n * c->n;
  hipLaunchKernelGGL(semh::k_hex_assemble, dim3(grid_for(total)), dim3(256), 0, st, H->d_map, vals,
                     total, out);
  HIP_TRY(hipGetLastError());
  return SEM_OK;
}

}  // namespace semh
