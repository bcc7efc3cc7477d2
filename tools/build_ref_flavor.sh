#!/bin/bash
# Build the library of a git revision as an A/B flavor:
#   bash tools/build_ref_flavor.sh <rev> <tag>  ->  ksim/libksim_engine_<tag>.so (KSIM_LIB_VARIANT=<tag>)
set -e
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" kube-scheduler-simulator_amd/csrc include | tar -x -C "$TMP"
make -C "$TMP/kube-scheduler-simulator_amd/csrc" -j8 OUT="$ROOT/kube-scheduler-simulator_amd/ksim/libksim_engine_$TAG.so" >/dev/null
rm -rf "$TMP"
