#!/bin/bash
# Host-side helper: build libathd.so of git revision REV (default HEAD) into OUT (default ablibs/libathd_prev.so)
# for whole-model A/B runs (tools/gpu_ab_lib.sh).  Usage: tools/build_rev.sh [REV] [OUT]
set -e
REV=${1:-HEAD}; OUT=$(realpath -m ${2:-ablibs/libathd_prev.so})
REPO=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/athd_rev.XXXX)
git -C "$REPO" archive "$REV" audio-to-sheet-music_amd/csrc include | tar -x -C "$W"
mkdir -p "$(dirname "$OUT")"
make -s -C "$W/audio-to-sheet-music_amd/csrc" -j8 OUT="$OUT" OBJDIR="$W/obj" > /dev/null
rm -rf "$W"
echo "$OUT"
