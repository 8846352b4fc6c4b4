#!/bin/bash
# r6: the inputs of the issue model (tools/issue_model.py).
#   issue_rate.txt: tools/_bin/issue_rate (tools/issue_rate.hip) on the GPU box
#   pmc_issue_c2.csv / pmc_issue_strips.csv + kernel_stats_*.csv: bash tools/pmc_issue.sh c2final,
#     bash tools/pmc_issue.sh stripsfinal --strips (one C2 pair / one strip batch alone)
#   *.s: python3 tools/issue_model.py --dump-isa profiles/r6/issue (the shipped library's ISA)
#   model.json / model.txt: python3 tools/issue_model.py --model --json profiles/r6/issue/model.json
set -o pipefail
timeout -k 10 300 tools/_bin/issue_rate > gpurun_out/r6d/issue_rate.txt 2>&1 &&
bash tools/pmc_issue.sh c2final && bash tools/pmc_issue.sh stripsfinal --strips
