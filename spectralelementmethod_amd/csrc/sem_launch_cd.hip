// Per-order launch unit of the Poisson column kernels with D as
// compile-time constants (DEOConst, csrc/deo_const.h), the
// orders n in [SEM_N_LO, SEM_N_HI].  A translation unit of its own: its
// compiler flags are chosen per order (_build.py LAUNCH_CD_FLAGS) without
// touching the argument-form kernels of sem_launch.hip.
#include "sem_ctx.h"

#ifndef SEM_N_LO
#define SEM_N_LO 2
#endif
#ifndef SEM_N_HI
#define SEM_N_HI 17
#endif

namespace semd {

template <int N>
void launch_poisson_const_d(const PoissonLaunch& L, bool nodal, bool seam, bool dot,
                            const WVec<N>& w, bool pat) {
  const DEO<N> D{};  // unused by the constant-D instantiations
  // the 16-bit map as a pattern table (MapRef, csrc/sem_kernels.h)
  if constexpr (PatternMap<N>::value) {
    if (pat) {
#define SEM_CD_LAUNCH_PAT(NODAL, SEAM, DOT)                                                  \
  hipLaunchKernelGGL((k_poisson_apply<N, NODAL, true, SEAM, DOT, true, true>), L.g, L.b, 0, L.st, \
                     L.mr, L.GP, L.XG, L.u, L.y, L.c0, L.c1, L.rounds, L.acc, D, w, L.sp)
      if (seam && dot) {
        if (nodal)
          SEM_CD_LAUNCH_PAT(true, true, true);
        else
          SEM_CD_LAUNCH_PAT(false, true, true);
      } else if (seam) {
        if (nodal)
          SEM_CD_LAUNCH_PAT(true, true, false);
        else
          SEM_CD_LAUNCH_PAT(false, true, false);
      } else {
        if (nodal)
          SEM_CD_LAUNCH_PAT(true, false, false);
        else
          SEM_CD_LAUNCH_PAT(false, false, false);
      }
#undef SEM_CD_LAUNCH_PAT
      return;
    }
  }
#define SEM_CD_LAUNCH(NODAL, SEAM, DOT)                                                       \
  hipLaunchKernelGGL((k_poisson_apply<N, NODAL, true, SEAM, DOT, true>), L.g, L.b, 0, L.st, L.mr, \
                     L.GP, L.XG, L.u, L.y, L.c0, L.c1, L.rounds, L.acc, D, w, L.sp)
  if (seam && dot) {
    if (nodal)
      SEM_CD_LAUNCH(true, true, true);
    else
      SEM_CD_LAUNCH(false, true, true);
  } else if (seam) {
    if (nodal)
      SEM_CD_LAUNCH(true, true, false);
    else
      SEM_CD_LAUNCH(false, true, false);
  } else {
    if (nodal)
      SEM_CD_LAUNCH(true, false, false);
    else
      SEM_CD_LAUNCH(false, false, false);
  }
#undef SEM_CD_LAUNCH
}

#define SEM_INSTANTIATE_CD(N)                                                               \
  template void launch_poisson_const_d<N>(const PoissonLaunch&, bool, bool, bool, const WVec<N>&, \
                                          bool);

#if SEM_N_LO <= 2 && 2 <= SEM_N_HI
SEM_INSTANTIATE_CD(2)
#endif
#if SEM_N_LO <= 3 && 3 <= SEM_N_HI
SEM_INSTANTIATE_CD(3)
#endif
#if SEM_N_LO <= 4 && 4 <= SEM_N_HI
SEM_INSTANTIATE_CD(4)
#endif
#if SEM_N_LO <= 5 && 5 <= SEM_N_HI
SEM_INSTANTIATE_CD(5)
#endif
#if SEM_N_LO <= 6 && 6 <= SEM_N_HI
SEM_INSTANTIATE_CD(6)
#endif
#if SEM_N_LO <= 7 && 7 <= SEM_N_HI
SEM_INSTANTIATE_CD(7)
#endif
#if SEM_N_LO <= 8 && 8 <= SEM_N_HI
SEM_INSTANTIATE_CD(8)
#endif
#if SEM_N_LO <= 9 && 9 <= SEM_N_HI
SEM_INSTANTIATE_CD(9)
#endif
#if SEM_N_LO <= 10 && 10 <= SEM_N_HI
SEM_INSTANTIATE_CD(10)
#endif
#if SEM_N_LO <= 11 && 11 <= SEM_N_HI
SEM_INSTANTIATE_CD(11)
#endif
#if SEM_N_LO <= 12 && 12 <= SEM_N_HI
SEM_INSTANTIATE_CD(12)
#endif
#if SEM_N_LO <= 13 && 13 <= SEM_N_HI
SEM_INSTANTIATE_CD(13)
#endif
#if SEM_N_LO <= 14 && 14 <= SEM_N_HI
SEM_INSTANTIATE_CD(14)
#endif
#if SEM_N_LO <= 15 && 15 <= SEM_N_HI
SEM_INSTANTIATE_CD(15)
#endif
#if SEM_N_LO <= 16 && 16 <= SEM_N_HI
SEM_INSTANTIATE_CD(16)
#endif
#if SEM_N_LO <= 17 && 17 <= SEM_N_HI
SEM_INSTANTIATE_CD(17)
#endif

}  // namespace semd
