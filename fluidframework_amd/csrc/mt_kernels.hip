// mt_kernels.hip — one capacity class of the replay, snapshot-load and generator kernels.
//
// Compiled once per class with -DMT_SEG=<segment slots> (kClassSegs in mt_device.h); each
// object exports mt_replay_kernel_<SEG>, mt_writer_kernel_<SEG>, mt_bigprops_kernel_<SEG>,
// mt_load_kernel_<SEG> and mt_generate_kernel_<SEG>,
// which mt_host.cpp selects per launch.  Keeping the class a template argument makes every LDS
// table base an immediate offset (mt::make_layout) instead of a runtime pointer.

#include "mt_engine.hip"

#ifndef MT_SEG
#error "compile with -DMT_SEG=<class>"
#endif

#define MT_CAT2(a, b) a##b
#define MT_CAT(a, b) MT_CAT2(a, b)

// The replay kernels' register budget: 512 / kWpe VGPRs.  The LDS classes allow the waves their
// layout lets a CU hold (mt_device.h class_waves_per_eu; -DMT_WPE_UNIFORM=4 gives every LDS class
// the 4-waves budget, the A/B baseline); the giant and HBM classes run one document per SIMD at most.
#ifdef MT_WPE_UNIFORM
constexpr int kWpe = mt::is_hbm_seg(MT_SEG) ? 1 : MT_WPE_UNIFORM;
#else
constexpr int kWpe = mt::class_waves_per_eu(MT_SEG);
#endif

// MT_PART (build parallelism): 1 = the observer replay and the generator, 2 = the writer, bigprops
// and load kernels; unset = all of them in one object
#if !defined(MT_PART) || MT_PART == 1
// the giant class's observer replay: the replaying wave plus its prefetch wave (mt_engine.hip giant_prefetch)
constexpr int kReplayThreads = mt::is_giant_seg(MT_SEG) ? mt::kGiantThreads : 64;
extern "C" __global__ __launch_bounds__(kReplayThreads) __attribute__((amdgpu_waves_per_eu(kWpe))) void MT_CAT(mt_replay_kernel_, MT_SEG)(mt::ReplayParams P) {
    mt::replay_body<MT_SEG, false>(P);
}

extern "C" __global__ __launch_bounds__(64) void MT_CAT(mt_generate_kernel_, MT_SEG)(mt::ReplayParams P) {
    mt::generate_body<MT_SEG>(P);
}
#endif

#if !defined(MT_PART) || MT_PART == 2
// writer replicas: the same replay plus the local-client path (local ops, pending segment groups,
// acks by the replica's own sequenced messages)
#ifdef MT_WRITER_WPE  // (A/B: the writer kernels' own register budget)
constexpr int kWriterWpe = kWpe > MT_WRITER_WPE ? MT_WRITER_WPE : kWpe;
#else
constexpr int kWriterWpe = kWpe;
#endif
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kWriterWpe))) void MT_CAT(mt_writer_kernel_, MT_SEG)(mt::ReplayParams P) {
    mt::replay_body<MT_SEG, false, true>(P);
}

// the observer replay with property sets of any size (props_extend_big): documents whose sets outgrow
// one pair per lane re-run here (cap_kind 3, mt_device.h kCapPool), so the replay kernels above carry none of it
// (the spill classes' replay kernels hold sets of any size themselves: the host never launches
// their bigprops kernel, whose body is empty)
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kWpe))) void MT_CAT(mt_bigprops_kernel_, MT_SEG)(mt::ReplayParams P) {
    if constexpr (!mt::is_hbm_seg(MT_SEG)) mt::replay_body<MT_SEG, false, false, true>(P);
}

// SnapshotLoader: the leading LOAD_HEADER / COLLAB / LOAD_BODY records of each document, then a
// checkpoint that the document's first replay launch resumes from
extern "C" __global__ __launch_bounds__(64) void MT_CAT(mt_load_kernel_, MT_SEG)(mt::ReplayParams P) {
    mt::replay_body<MT_SEG, true>(P);
}
#endif
