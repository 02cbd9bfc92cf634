#!/bin/bash
# Round 4 (k): measurement cycle with the shadow-map bin split A/B (parts1 = one workgroup per map bin), then the
# per-rank band costs at 3 frames in flight (tools/sim_bands.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TRACE_CFGS="c3 c5" bash tools/gpu_cycle.sh parts1 && INFLIGHT=3 bash tools/sim_bands.sh
