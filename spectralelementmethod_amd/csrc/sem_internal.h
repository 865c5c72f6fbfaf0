// Internal declarations shared by the host (sem_basis.cpp) and device
// (sem_device.hip) halves of libsem_hip.so.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/sem_hip.h"

#define SEM_MAX_ORDER 16
#define SEM_MAXN (SEM_MAX_ORDER + 1)

namespace sem {

// thread-local error message behind sem_last_error()
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

// host basis helpers (sem_basis.cpp)
int gll_table(int p, double* nodes, double* bary, double* quad);
void diff_matrix(int n, const double* nodes, const double* bary, double* D);
void lagrange_eval(int n, const double* nodes, const double* bary, int64_t nx, const double* x,
                   double* B);
int invert(int n, const double* A, double* Ainv);

}  // namespace sem

// accessors of the operator context for the domain-decomposition layer
// (sem_dd.hip)
namespace sem {
int64_t ctx_ndof(const sem_ctx* c);
int ctx_device(const sem_ctx* c);
// bumped by every call that changes what a launch reads (map, geometry,
// basis, modes, Reynolds number, linearisation buffer): a captured step
// compares it before replaying (sem_dd.hip)
uint64_t ctx_epoch(const sem_ctx* c);
// nodes the context zeroes before an overwrite (its zero list) copied to the
// host; *only_unreferenced: the list holds only nodes none of the context's
// elements touch (no atomic first writers), so zeroing them may be deferred
// to any later kernel on the same stream
int ctx_zero_list(const sem_ctx* c, std::vector<uint32_t>* nodes, bool* only_unreferenced);
int ctx_dpn(const sem_ctx* c);
// bumped by sem_set_map_shared only (the plan, hence the zero list, changed)
uint64_t ctx_map_epoch(const sem_ctx* c);

// The decomposition's finish fused with the interior context's seam sum
// (sem_dd.hip): one launch that writes every seam node of the interior
// (y[g] = its colour slots, as k_seam_sum) plus, for a seam node the
// interface also touches, the interface value and the neighbours' values;
// then the remaining interface DOFs and the deferred zero list as k_dd_finish.
struct DDFinish {
  const uint32_t* fidx;  // [nc] local DOF | overwrite << 31
  int64_t nc;
  const double* yc;      // interface values (indexed like y when yc_local)
  int yc_local;
  const int32_t* rp;     // [nc + 1] received values of compact DOF j at rpos[rp[j]..)
  const uint32_t* rpos;
  const double* recv;
  const uint32_t* fzero;  // DOFs to zero
  int64_t nz;
  const int32_t* seam_cj;  // [n_seam] compact DOF of the seam node, or -1
  const uint32_t* rest;    // compact DOFs that are not seam nodes
  int64_t n_rest;
  // split finish (sem_dd.hip dd_finish): sel = the seam nodes this launch
  // handles (null: all); rest handled unless skip_rest, the zero list
  // unless skip_zero
  const uint32_t* sel = nullptr;
  int64_t n_sel = 0;
  int skip_rest = 0, skip_zero = 0;
};
// seam plan of a one-DOF-per-node context: true when sem_apply can leave its
// seam sum to ctx_seam_finish; the seam nodes' ids copied to the host
bool ctx_seam_fusable(const sem_ctx* c);
int ctx_seam_gids(const sem_ctx* c, std::vector<uint32_t>* gids);
void ctx_set_defer_seam_sum(sem_ctx* c, bool defer);
int ctx_seam_finish(sem_ctx* c, double* y, const DDFinish& f, hipStream_t st);
// any seam node with a prior value (SEM_NODE_PRIOR): such a plan is not
// fused with the pack
bool ctx_seam_has_prior(const sem_ctx* c);
// the context's seam sum (deferred by sem_apply) fused with the pack of
// send[k] = y[sidx[k]], k < ne (sj[k]: seam index of that DOF, or -1)
int ctx_seam_pack(sem_ctx* c, double* y, double* send, const uint32_t* sidx, const int32_t* sj,
                  int64_t ne, hipStream_t st);
}  // namespace sem
