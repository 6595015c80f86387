#!/bin/bash
# Background GPU call with transient-retry (tools/gpu.sh); output in /tmp/gpurun_bg.log.
GPU_TIMEOUT=${GPU_TIMEOUT:-900} nohup tools/gpu.sh "$@" > /tmp/gpurun_bg.log 2>&1 &
echo "started pid $!"
