#!/bin/bash
# Builds cost-experiment variants of libsgn (NOT parity-valid): ../libsgn_exp_<name>.so
# usage: bash build_exp.sh name "-DFLAG ..."
set -e
cd "$(dirname "$0")"
HIPCC=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value -I../../include -I."
$HIPCC $F $2 -c engine.hip -o engine_exp_$1.o
$HIPCC --offload-arch=gfx950 -shared -o ../libsgn_exp_$1.so api.o routes.o engine_exp_$1.o frontend.o comm.o pcap.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
