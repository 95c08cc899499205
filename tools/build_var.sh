#!/bin/bash
# Experiment build of the backend restricted to the C3 kernels (-DMODEM_DEV_MIN), plus any
# extra flags, into rust-modem_amd/build/var/<name>/libmodem_hip.so (A/B with tools/ab.sh).
# FULL=1: every kernel variant (no -DMODEM_DEV_MIN), as the in-tree library.
# Usage: [FULL=1] tools/build_var.sh <name> [hipcc flags...]
set -e
name=$1; shift
cd "$(dirname "$0")/../rust-modem_amd"
d=build/var/$name; mkdir -p $d
DEVMIN=-DMODEM_DEV_MIN; [ "${FULL:-0}" = 1 ] && DEVMIN=
for f in tx rx chain misc; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 $DEVMIN "$@" \
    -c csrc/modem_$f.hip -o $d/$f.o &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $DEVMIN "$@" -x hip -c csrc/modem_capi.cpp -o $d/c.o &
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $d/tx.o $d/rx.o $d/chain.o $d/misc.o $d/c.o -o $d/libmodem_hip.so
echo "built $d/libmodem_hip.so"
