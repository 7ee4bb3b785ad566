#!/bin/bash
# round 3: profiles of the build (kernel stats, PMC traffic, HIP API trace) for cfg2/cfg4/cfg5,
# SQ counters of the cfg2 int8 kernel
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=r3k bash tools/profile_all.sh stats pmc api cfg4 cfg5 || exit $?
TAG=r3k bash tools/pmc_sq2.sh
