#!/bin/bash
# round-4 gate, call 2: rocprofv3 kernel statistics of the S-A and S-C bench commands (the
# roofline kernel's mean duration beside the bench line's HIP-event figure), the per-tick band
# times of the S-A schedule, and the FAITHFUL wall times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu.sh r04h prof_sa prof_sc ticks faithful prof_faithful
