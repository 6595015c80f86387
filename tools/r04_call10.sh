#!/bin/bash
# Round-4 closing evidence: rocprofv3 traces / PMC (tools/r04_evidence.sh), then the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r04_evidence.sh gpurun_out/r04_evidence > gpurun_out/r04_evidence.log 2>&1 || exit $?
