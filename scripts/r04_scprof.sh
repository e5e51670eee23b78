#!/bin/bash
# round-4 end: rocprof kernel statistics and the SQ instruction mix of the S-C bench with the
# late round-4 tick kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu.sh r04zi prof_sc mix_sc
