#!/bin/bash
# round 3 final build (merge registers): kernel stats, PMC traffic, HIP API trace (cfg2/cfg4/cfg5), SQ counters
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=r3t bash tools/profile_all.sh stats pmc api cfg4 cfg5 || exit $?
TAG=r3t bash tools/pmc_sq2.sh
