#!/bin/bash
# Build an A/B tree DIR from SRC (a tree) with extra compiler flags for libgpd.so.
# usage: tools/ab_flags_build.sh SRC DIR "flags"
set -eu
SRC=$1; D=$2; FL=$3
rm -rf "$D"; mkdir -p "$D"
(cd "$SRC" && tar --exclude=./.git --exclude=./gpurun_out --exclude=./profiles --exclude='./ab_*' \
    --exclude='*.so' --exclude=__pycache__ -cf - .) | tar -C "$D" -xf -
(cd "$D" && GPD_EXTRA_CFLAGS="$FL" python -c "from gopacket_amd.build import build_lib, build_synth, build_oracle; build_lib(force=True); build_synth(); build_oracle()")
echo "built $D ($FL)"
