#!/bin/bash
# Builds cost-experiment variants of libsgn (NOT parity-valid): ../libsgn_exp_<name>.so
# usage: bash build_exp.sh name "-DFLAG ..."
set -e
cd "$(dirname "$0")"
HIPCC=/opt/rocm/bin/hipcc
# the variant links the product's other objects: rebuild them first, so every object of the
# variant was compiled against the same sgn_internal.h (round 5: a variant linked against stale
# objects segfaulted the host process; sgn_create now also refuses such a library)
make -s -j8 ../libsgn.so
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value -I../../include -I."
$HIPCC $F $2 -c engine.hip -o engine_exp_$1.o
$HIPCC --offload-arch=gfx950 -shared -o ../libsgn_exp_$1.so api.o routes.o engine_exp_$1.o frontend.o comm.o pcap.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
