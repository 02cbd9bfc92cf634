#!/bin/bash
# Frames in flight A/B on the bench (every config at 2, 3 and 4, then the defaults), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for rep in 1 2; do
  for n in 2 3 4; do echo "inflight $n"; EXTRA="--inflight $n" bash tools/ab.sh "" || exit 1; done
  echo "defaults"; bash tools/ab.sh "" || exit 1
done
