#!/bin/bash
# Round 6: TGEN host slots dealt over their kind's waves (SGN_HOST_ORDER=mix) against the
# bandwidth-sorted default, config C, same build, interleaved.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
bash tools/ab_env.sh C 3 "-" "SGN_HOST_ORDER=mix" || exit 1
echo DONE
