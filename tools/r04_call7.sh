#!/bin/bash
# One GPU call: gradient tests + variants, the loss-kernel regression hunt, the in-launch reduction A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r04_grad.sh > gpurun_out/grad.log 2>&1 || exit $?
bash tools/r04_regress.sh > gpurun_out/regress.log 2>&1 || exit $?
