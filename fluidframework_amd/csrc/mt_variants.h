// mt_variants.h -- every kernel-template instantiation libmtreplay.so launches, as
// X(name, kernel).  fluidframework_amd/build.py compiles each into a translation unit of its
// own that defines `const void *mtk_<name>()` (the kernel's host pointer); the host side
// (mt_replay.hip) launches through those pointers with hipLaunchKernel, so the ~25 large
// kernels compile in parallel.  -DMT_SINGLE_TU (build.py MT_SINGLE_TU=1) defines them in
// mt_replay.hip instead.
#pragma once
#define MT_VARIANTS(X)                                                               \
    X(R_LDS_LOG, (k_replay<TierLdsT<true>, 1>))                                      \
    X(R_LDS, (k_replay<TierLdsT<false>, 1>))                                         \
    X(R_LDS2, (k_replay<TierLdsT<false>, 2>))                                        \
    X(R_LIVELDS_LOG, (k_replay<TierLiveLdsT<true>, 1>))                              \
    X(R_LIVELDS, (k_replay<TierLiveLdsT<false>, 1>))                                 \
    X(R_LIVE_LOG, (k_replay<TierLiveT<true>, 1>))                                    \
    X(R_LIVE, (k_replay<TierLiveT<false>, 1>))                                       \
    X(R_GLB_LOG, (k_replay<TierGlbT<true>, 1>))                                      \
    X(R_GLB, (k_replay<TierGlbT<false>, 1>))                                         \
    X(P_C3, (k_replay_paged<TierPagedT<false, true, false, false, 192, 192, 220>>))  \
    X(P_C4, (k_replay_paged<TierPagedT<false, false, false, true, 224, 900, 1900>>)) \
    X(P_PACKED_LOG, (k_replay_paged<TierPagedT<true, false, false, true>>))          \
    X(P_PACKED, (k_replay_paged<TierPagedT<false, false, false, true>>))             \
    X(P_BIG_LOG, (k_replay_paged<TierPagedT<true, false, true>>))                    \
    X(P_BIG, (k_replay_paged<TierPagedT<false, false, true>>))                       \
    X(P_NARROW_LOG, (k_replay_paged<TierPagedT<true, true>>))                        \
    X(P_LOG, (k_replay_paged<TierPagedT<true>>))                                     \
    X(P_NARROW, (k_replay_paged<TierPagedT<false, true>>))                           \
    X(P_FULL, (k_replay_paged<TierPagedT<false>>))                                   \
    X(P_HM, (k_replay_paged<TierPagedT<false, false, false, false, 0, 0, 0, true>>)) \
    X(P_BIG_HM, (k_replay_paged<TierPagedT<false, false, true, false, 0, 0, 0, true>>)) \
    X(P_HM_LOG, (k_replay_paged<TierPagedT<true, false, false, false, 0, 0, 0, true>>)) \
    X(P_BIG_HM_LOG, (k_replay_paged<TierPagedT<true, false, true, false, 0, 0, 0, true>>)) \
    X(G_LDS, (k_generate<TierLdsT<false>>))                                          \
    X(G_GLB, (k_generate<TierGlbT<false>>))                                          \
    X(GP_NARROW, (k_generate_paged<TierPagedT<false, true>>))                        \
    X(GP_FULL, (k_generate_paged<TierPagedT<false>>))                                \
    X(LC_FAST, (k_load_convert<TierPagedT<false>>))                                  \
    X(LC_LOG, (k_load_convert<TierPagedT<true>>))

#define MT_VARIANT_DECL(n, k) const void *mtk_##n();
MT_VARIANTS(MT_VARIANT_DECL)
#define MTK(n) mtk_##n()
