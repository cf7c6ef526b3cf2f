#!/bin/bash
# Copy a gpurun_out/prof_<tag> profile into profiles/<round>/<name>/ (flat CSV names), here.
#   tools/save_profile.sh gpurun_out/prof_v2 r01/c3_v2
set -e
SRC=$1; DST=profiles/$2
mkdir -p $DST
cp $SRC/kernel_stats.txt $SRC/pmc_traffic.json $SRC/bench_under_trace.json $DST/ 2>/dev/null || true
for d in $SRC/*/; do
  n=$(basename $d)
  for f in $(find $d -name "*.csv"); do
    b=$(basename $f | sed 's/^[0-9]*_//')
    cp $f $DST/${n}_$b
  done
done
ls $DST
