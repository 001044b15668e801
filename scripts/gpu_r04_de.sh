#!/bin/bash
# Round 4: gpu_r04_d.sh (parity + the scan-sums C1 A/B) then gpu_r04_e.sh (cache-policy A/Bs).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r04_d.sh && bash scripts/gpu_r04_e.sh
