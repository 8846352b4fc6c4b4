#!/bin/bash
# r6: what a fifth k_warp_iter block per CU is worth now (the issue model says the launch is
# issue- and latency-bound at 4 waves/SIMD).  tools/wi_probe.hip built twice:
#   wi_probe_m6_w0: the shipped margin 6 (39,936 B LDS, 97 VGPRs: 4 blocks/CU)
#   wi_probe_m4_w5: margin 4 (29,952 B) + amdgpu_waves_per_eu(5) (96 VGPRs): 5 blocks/CU
# (hipcc ... -DWI_M=<m> [-DWI_WPE=5] tools/wi_probe.hip), alternated twice per geometry.
set -o pipefail
for g in "6144 4096" "3146 2097"; do for b in m6_w0 m4_w5 m6_w0 m4_w5; do
  echo "== $b $g"; timeout -k 10 120 tools/_bin/wi_probe_$b $g 20 || exit 1
done; done
