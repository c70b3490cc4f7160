#!/bin/bash
# round-3 batch A: fp8 wgrad (tests + bench + dsv3 ABBA), then the headline profile + proxy
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r3_fp8wg.sh && bash tools/gpu/r3_prof_headline.sh
