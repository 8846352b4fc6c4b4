// The streaming and blocked iteration passes (k_iterate_roll, k_iterate_tb4, kb_iterate_roll),
// instantiated in their own translation unit so that they can be compiled with the
// instruction scheduler that suits them: the Makefile builds this file with
// -mllvm -amdgpu-sched-strategy=max-ilp (the default occupancy-first scheduler for
// tvl1_engine.hip, whose k_warp_iter would lose occupancy under max-ilp: 97 -> 184 VGPRs).
// Measured on one C2 pair (rocprofv3 kernel trace, two boxes, profiles/r3/ab_sched_ilp.txt):
// k_iterate_roll<4,2> 329 -> 300 and 334 -> 322 us, k_iterate_tb4 88.2 -> 82.9 and 89.4 -> 86.7
// us per launch, the same occupancy (189 VGPRs, 2 SGPRs spilled); C2 +1.2 %, production
// strips +2.2 % (A/B in one call).  The arithmetic is the same operations in the same order,
// so the same bits (-ffp-contract=off; the whole -m gpu suite passes on this build).
// tvl1_engine.hip declares every instantiation below `extern template` (TVL1_PASS_INSTANCES).
#define TVL1_PASSES_TU 1
#include "tvl1_kernels.hpp"
#include "tvl1_batch.hpp"

namespace tvl1k {
#define TVL1_PASS_INSTANCE(...) template __global__ void __VA_ARGS__;
#include "tvl1_passes.inc"
#undef TVL1_PASS_INSTANCE
}  // namespace tvl1k
