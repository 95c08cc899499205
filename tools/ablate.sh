#!/bin/bash
# Build ablation variants of the backend (profiling only) into rust-modem_amd/build/ablate/<v>/.
# Each variant drops one stage of the kernels so its cost shows up as a time difference.
# TX (-DMODEM_ABLATE_<v>): FIR (no matrix products), TRIG (no sin/cos), MIX (no carrier mix),
# STORE (no output stores). RX (-DMODEM_RX_ABLATE_<v>): RX_LOAD (no sample loads), RX_FIR
# (no matched filter), RX_STORE (no output stores). Usage: tools/ablate.sh [variants...]
set -e
cd "$(dirname "$0")/../rust-modem_amd"
vars=${@:-base FIR TRIG MIX STORE RX_LOAD RX_FIR RX_STORE}
for v in $vars; do
  d=build/ablate/$v; mkdir -p $d
  case $v in
    base) extra="" ;;
    RX_*) extra="-DMODEM_RX_ABLATE_${v#RX_}" ;;
    *) extra="-DMODEM_ABLATE_$v" ;;
  esac
  for f in tx rx misc; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 $extra -c csrc/modem_$f.hip -o $d/$f.o &
  done
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -x hip -c csrc/modem_capi.cpp -o $d/c.o &
done
wait
for v in $vars; do
  d=build/ablate/$v
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $d/tx.o $d/rx.o $d/misc.o $d/c.o -o $d/libmodem_hip.so
done
