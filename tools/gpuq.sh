#!/bin/bash
# retry gpurun while no GPU slot/box is free (rc 3: nothing ran, nothing charged)
out=$1; shift; lim=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $lim -- "$@" > $out 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $out; then echo "rc=$rc" >> $out; exit $rc; fi
  sleep 90
done
echo "gave up" >> $out
