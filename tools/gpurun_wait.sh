#!/bin/bash
# gpurun, waiting for a free slot: when the pool answers "busy / no box free" (nothing ran, nothing
# charged) the same call is made again after a pause, up to TRIES times. Any call that ran — pass
# or fail — is returned as it is (never retried). Usage: tools/gpurun_wait.sh LOG TIMEOUT 'cmd'
LOG=$1; T=$2; CMD=$3
for i in $(seq ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "nothing was charged\|no free box\|stopped responding while being prepared" "$LOG" \
      && ! grep -q "status=ok\|status=fail" "$LOG"; then
    sleep ${PAUSE:-90}
    continue
  fi
  exit $rc
done
exit 3
