#!/bin/bash
# r06f: drop-in encode kernel: write-through stores vs the mailbox tree (tools/mailbox_probe);
# CRC64 checksum-only bench at the per-pass geometry.
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O; cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for f in nt-sync sc1nt-sync nt-tree sc1nt-tree; do
    timeout -k 10 60 ./tools/mailbox_probe $f 3000 >> $O/wall.jsonl 2>> $O/wall.err || { tail $O/wall.err; exit 1; }
  done
done
cat $O/wall.jsonl
for f in nt-sync sc1nt-sync nt-tree sc1nt-tree; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$f -o kt -- ./tools/mailbox_probe $f 1000 > $O/kt_$f.log 2>&1 || { tail $O/kt_$f.log; exit 1; }
done
timeout -k 10 300 python bench.py --workload crc64 --no-cpu-baseline > $O/bench_crc64.json 2> $O/bench_crc64.err || { tail $O/bench_crc64.err; exit 1; }
cat $O/bench_crc64.json
