#!/bin/bash
# Same-box A/B of the speculative gather width (SGN_GATHER_SPEC) on configs B and D
set -u
for rep in 1 2 3; do
  for v in 16 64 32; do bash tools/exp_env.sh B_g${v}_$rep B SGN_GATHER_SPEC=$v || exit 1; done
  for v in 16 64; do bash tools/exp_env.sh D_g${v}_$rep D SGN_GATHER_SPEC=$v || exit 1; done
done
