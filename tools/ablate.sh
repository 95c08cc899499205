#!/bin/bash
# Build ablation variants of the backend (profiling only) into rust-modem_amd/build/ablate/<v>/.
# Each variant drops one stage of the kernels so its cost shows up as a time difference.
set -e
cd "$(dirname "$0")/../rust-modem_amd"
for v in base FIR TRIG MIX STORE; do
  d=build/ablate/$v; mkdir -p $d
  extra=""; [ "$v" != base ] && extra="-DMODEM_ABLATE_$v"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 $extra -c csrc/modem_kernels.hip -o $d/k.o &
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -x hip -c csrc/modem_capi.cpp -o $d/c.o &
  wait
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $d/k.o $d/c.o -o $d/libmodem_hip.so
done
