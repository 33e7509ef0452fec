#!/bin/bash
# Same-box A/B of the bench (no CPU leg) between libsgn and experiment variants, alternating
# twice. usage: r04_ab.sh <tag> <workload> <steps> <variant>...   (variant "base" = libsgn.so)
set -u
T=$1; W=$2; S=$3; shift 3
for rep in 1 2; do
  for v in "$@"; do
    bash tools/exp_one.sh $v $W ${T}_$rep --steps $S --warmup 5 || exit 1
  done
done
