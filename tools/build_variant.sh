#!/bin/bash
# Build a variant of the extension for a kernel A/B or a profiling run, on the CPU container:
#   tools/build_variant.sh NAME [device flags...]   ->  ab/_C_NAME.so
# e.g. tools/build_variant.sh stamp -DSPA_DKDV3_STAMP=1; run it on the GPU box with
#   SPA_EXT_SO=ab/_C_stamp.so SPA_ATTN_STAMP=1 python tools/bench_attn.py ...
# (objects under build/NAME; the in-tree solvingpapers_amd/_C.so is not touched)
set -eo pipefail
name=${1:?variant name}; shift
cd "$(dirname "$0")/.."
SPA_BUILD_VARIANT=$name SPA_BUILD_DEFINES="$*" python -m solvingpapers_amd._build
