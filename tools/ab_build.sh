#!/bin/bash
# Build an A/B variant package: ab/<name>/toymeshpathtracer_amd with its own
# libtmpt.so compiled with EXTRA flags (tools/ab_kpath.py runs it against ".").
# usage: bash tools/ab_build.sh <name> "<extra flags>"
set -e
name=$1; extra=$2
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/ab/$name/toymeshpathtracer_amd
mkdir -p $dst
cp $root/toymeshpathtracer_amd/*.py $dst/
make -s -C $root/toymeshpathtracer_amd/csrc -j8 OUTDIR=$dst/_lib EXTRA="$extra" $dst/_lib/libtmpt.so
echo "built $dst ($extra)"
