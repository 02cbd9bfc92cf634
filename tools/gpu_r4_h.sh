#!/bin/bash
# Round 4 (h): measurement cycle with the texel-pair A/B (texture, map and sky pairs off), then the full bench line
# at 2 and 3 frames in flight (tools/gpu_misc2.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_cycle.sh nopairs && bash tools/gpu_misc2.sh
