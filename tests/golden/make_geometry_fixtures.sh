#!/usr/bin/env bash
# Regenerates tests/golden/example_geometry.bin from the reference's own layout parser
# (parseLayout.c:359, run on /root/reference/example.png at the default 30 px/m of main.c:26, TILE_SIZE
# 200 of main.c:44) via oracle/_ref/dump_geometry (built by oracle/build_ref.sh). Run in this
# container (needs /root/reference); the .bin is committed so the GPU box never needs the reference.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(dirname "$(dirname "$HERE")")"
bash "$REPO/oracle/build_ref.sh"
TMP=$(mktemp -d)
( cd "$TMP" && "$REPO/oracle/_ref/dump_geometry" /root/reference/example.png 30 "$HERE/example_geometry.bin" )
rm -rf "$TMP"
