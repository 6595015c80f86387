#!/bin/bash
# Submit one gpurun call; re-submit only when the infrastructure reports a transient failure
# (status "transient": nothing ran, nothing charged).  Never retries a command that ran.
T=${GPU_TIMEOUT:-900}
for attempt in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[gpu.sh] transient infrastructure failure (attempt $attempt); waiting 45 s"
  sleep 60
done
exit 1
