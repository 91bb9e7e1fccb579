#!/bin/bash
# Submit one gpurun call, re-submitting it ONLY while the pool reports an
# infrastructure transient (nothing ran, nothing charged: busy slots, no box,
# a box lost while being prepared, backoff). Any call that actually ran —
# pass or fail — ends the loop; a failing GPU step is never re-run.
#   tools/gpurun_when_free.sh <timeout_s> <log> <command...>
T=$1; LOG=$2; shift 2
for attempt in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then echo "attempt $attempt status=$st" >> "$LOG"; exit 0; fi
  wait_s=$(python3 -c "
import json,re
m=json.load(open('gpurun_out/.last_call.json')).get('msg','')
r=re.search(r'retry in (\d+)s',m)
print(int(r.group(1))+15 if r else 90)" 2>/dev/null)
  sleep "${wait_s:-90}"
done
echo "gave up after 40 transients" >> "$LOG"
