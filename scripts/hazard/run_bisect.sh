#!/bin/bash
# run every bisect build; print the branchy total line per opt-bisect-limit
for f in scripts/hazard/bisect/ph_*; do
  out=$(timeout -k 5 60 $f | tail -1); rc=$?
  echo "$(basename $f) rc=$rc $out"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
