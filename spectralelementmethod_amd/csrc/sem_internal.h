// Internal declarations shared by the host (sem_basis.cpp) and device
// (sem_device.hip) halves of libsem_hip.so.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

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
}  // namespace sem
