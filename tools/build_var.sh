#!/bin/bash
# Experiment build of the backend into rust-modem_amd/build/var/<name>/libmodem_hip.so (A/B with
# tools/ab.sh, tools/ab_variants.sh), with the MODEM_VARIANTS_MIN build option (modem_variants.h:
# the BASELINE filters' matrix-core variants only; other filters run on the VALU kernels) plus any
# extra hipcc flags. FULL=1: every variant, as the in-tree library.
# Usage: [FULL=1] tools/build_var.sh <name> [hipcc flags...]
set -e
name=$1; shift
cd "$(dirname "$0")/../rust-modem_amd"
d=build/var/$name; mkdir -p $d
MIN=-DMODEM_VARIANTS_MIN; [ "${FULL:-0}" = 1 ] && MIN=
srcs="tx rx chain misc txm_f32 txm_f16 txm_bb txm_real rxm_f32 rxm_f16 rxm_mixed"
for f in $srcs; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form=1 --offload-arch=gfx950 $MIN "$@" \
    -c csrc/modem_$f.hip -o $d/$f.o &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $MIN "$@" -x hip -c csrc/modem_capi.cpp -o $d/c.o &
wait
objs=""; for f in $srcs; do objs="$objs $d/$f.o"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $d/c.o -o $d/libmodem_hip.so
echo "built $d/libmodem_hip.so"
