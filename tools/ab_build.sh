#!/bin/bash
# Build libacehip.so from a git revision (or the working tree: rev "WT") with
# optional extra compiler flags into tools/ab/libacehip_<tag>.so, for in-process
# A/B benchmarking (MI355X timings vary ±10-20 % between boxes, so comparisons
# must share one process).
# usage: tools/ab_build.sh <rev|WT> <tag> ["-DFOO=1 ..."]
set -e
REV=${1:-HEAD}; TAG=${2:-ref}; EXTRA=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
if [ "$REV" = "WT" ]; then
    mkdir -p "$W/ace-step-1.5_amd" && cp -r "$ROOT/ace-step-1.5_amd/csrc" "$ROOT/ace-step-1.5_amd/Makefile" "$W/ace-step-1.5_amd/"
    cp -r "$ROOT/include" "$W/"
else
    git -C "$ROOT" archive "$REV" ace-step-1.5_amd/csrc ace-step-1.5_amd/Makefile include | tar -x -C "$W"
fi
mkdir -p "$W/ace-step-1.5_amd/acehip"
make -C "$W/ace-step-1.5_amd" -j8 EXTRA="$EXTRA" >/dev/null
mkdir -p "$ROOT/tools/ab"
cp "$W/ace-step-1.5_amd/acehip/libacehip.so" "$ROOT/tools/ab/libacehip_$TAG.so"
rm -rf "$W"
echo "built tools/ab/libacehip_$TAG.so from $REV $EXTRA"
