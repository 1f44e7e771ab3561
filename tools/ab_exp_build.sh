#!/bin/bash
# Build A/B variant trees ab_e<N>/ (a copy of the working tree whose libgpd.so is compiled with
# -DGPD_EXP=<N>, gpd_kernels.hip kExp* bits) for tools/ab_exp.sh.  Runs on the CPU container.
# usage: tools/ab_exp_build.sh N [N ...]
set -eu
cd "$(dirname "$0")/.."
for N in "$@"; do
  D=ab_e$N
  rm -rf "$D"; mkdir -p "$D"
  tar --exclude=./.git --exclude=./gpurun_out --exclude=./profiles --exclude='./ab_*' \
      --exclude='*.so' --exclude=__pycache__ --exclude=./build -cf - . | tar -C "$D" -xf -
  (cd "$D" && GPD_EXTRA_CFLAGS="-DGPD_EXP=$N" python -c "from gopacket_amd.build import build_lib, build_synth, build_oracle; build_lib(force=True); build_synth(); build_oracle()")
  echo "built $D"
done
