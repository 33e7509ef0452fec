#!/bin/bash
# Same-box A/B of libsgn variants: r03_ab.sh <tag> "<variants>" "<workloads>" [bench args]
# (variants: base = libsgn.so, else libsgn_exp_<v>.so; each workload alternates the variants twice)
set -u
T=$1; VS=$2; WS=$3; shift 3
for w in $WS; do
  for rep in 1 2; do
    for v in $VS; do bash tools/exp_one.sh $v $w ${T}r$rep "$@" || exit 1; done
  done
done
