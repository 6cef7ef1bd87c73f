set -o pipefail
cd /root/repo
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for e in X=1 ORION_ATTN_XCD=0; do
  for shp in "64 1024 12 12 64" "4 4096 32 32 128"; do
    d=gpurun_out/trab/$(echo $e | tr '=' '_')_$(echo $shp | tr ' ' '_')
    mkdir -p $d
    (cd /tmp && env $e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$d -o t -- python3 /root/repo/scripts/attn_one.py $shp 5 > /root/repo/$d/log 2>&1) || exit 1
    f=$(find $d -name '*kernel_stats.csv' | head -1)
    echo "== $e $shp"
    python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'attn' in r['Name']: print('  %-50s %8.1f us' % (r['Name'][:50], float(r['AverageNs'])/1e3))"
  done
done
