#!/bin/bash
# round 3 final build: kernel stats, PMC traffic, HIP API trace (cfg2/cfg4/cfg5), SQ counters
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=r3r bash tools/profile_all.sh stats pmc api cfg4 cfg5 || exit $?
TAG=r3r bash tools/pmc_sq2.sh
