#!/bin/bash
# Round 6: which workgroup serves which host group (SGN_GROUP_ROT: TGEN server groups on the
# workgroups dispatched in the 4th pass, alone on their SIMD if dispatch is round-robin), C.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for i in 1 2; do
bash tools/ab_env.sh C 1 "-" "SGN_GROUP_ROT=768" || exit 1
bash tools/ab_env.sh C 1 "SGN_GROUP_ROT=512" "SGN_GROUP_ROT=1024" || exit 1
done
echo DONE
