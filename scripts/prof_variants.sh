#!/bin/bash
# rocprofv3 kernel stats of bench.py for each named variant: prof_variants.sh NAME [NAME ...]
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in "$@"; do
  ADMM_TOMO_LIB=variants/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profv_$v -o run \
    --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --strong none > gpurun_out/profv_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/profv_$v -name "*kernel_stats.csv" | head -1)
  python - "$f" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(sys.argv[2], r["Name"][:48].ljust(48), r["Calls"].rjust(5), "%.2f us" % (float(r["AverageNs"]) / 1e3))
PY
done
