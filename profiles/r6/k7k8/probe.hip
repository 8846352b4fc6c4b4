#define TVL1_PASSES_TU 1
#include "tvl1_kernels.hpp"
#include "tvl1_batch.hpp"
namespace tvl1k {
template __global__ void kb_iterate_roll<4, 2, 0>(BatchRoll);
template __global__ void kb_iterate_roll<6, 2, 0>(BatchRoll);
template __global__ void kb_iterate_roll<7, 2, 0>(BatchRoll);
template __global__ void kb_iterate_roll<8, 2, 0>(BatchRoll);
}
