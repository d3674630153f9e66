#!/bin/bash
# Round 4, calls k + l in one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4l.sh && bash tools/gpu_r4k.sh
