#!/bin/bash
# Kernel stats of the A/B main-pass forms at C2 (k_tokenize's own time in the split forms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02u
GM_MATCH_MAIN=coop bash scripts/kstats.sh r02u_coop --steps 3 --warmup 1 --no-cpu --no-parity --no-host-io | tee gpurun_out/r02u/coop.txt || exit 1
GM_MATCH_MAIN=split bash scripts/kstats.sh r02u_split --steps 3 --warmup 1 --no-cpu --no-parity --no-host-io | tee gpurun_out/r02u/split.txt || exit 1
