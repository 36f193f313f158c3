#!/bin/bash
# kernel profiles (rocprofv3 --kernel-trace --stats, csv) of the driver's C2 command at given workloads
#   bench_tools/r04_prof.sh OUTDIR "name:args" ...
set -o pipefail
OUT=$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
X="${PROF_X:---steps 20 --warmup 2} --no-cpu-baseline --no-host-buffers --collector-windows 0 --sustained-steps 0"
for v in "$@"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$name -o run -- python3 -u bench.py $X $a > $OUT/prof_$name.json 2> $OUT/prof_$name.err || { echo "prof $name failed"; tail -5 $OUT/prof_$name.err; exit 1; }
  f=$(find $OUT/prof_$name -name "*kernel_stats.csv" | head -1); cp $f $OUT/${name}_kernel_stats.csv
  python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/${name}_kernel_stats.csv')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
print('== $name')
for r in rows[:14]: print('%-40s calls %6s avg_us %9.1f total_ms %8.1f pct %5.1f' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6, float(r['Percentage'])))
"
  find $OUT/prof_$name -name "*.csv" ! -name "*kernel_stats.csv" -delete
done
