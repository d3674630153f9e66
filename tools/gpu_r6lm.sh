#!/bin/bash
# Round 6, calls l + m in one lease.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r6l.sh; rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
bash tools/gpu_r6m.sh
