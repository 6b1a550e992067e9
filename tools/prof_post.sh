#!/bin/bash
# On the GPU box, after a profile set: per-kernel summaries of every kernel trace (profdb.py, ms/step
# over the traced steps, and the idle-gap timeline), then gzip every trace .db and PMC CSV so the
# call's gpurun_out/ stays under the 64 MiB copy-back limit.
# usage: bash tools/prof_post.sh <tag>
T=${1:?tag}
cd $GRAFT_REPO_ROOT
for d in gpurun_out/${T}_prof_*/ gpurun_out/${T}_prof/; do
  [ -d "$d" ] || continue
  db=$(ls "$d"*.db 2>/dev/null | head -1)
  [ -n "$db" ] || continue
  n=$(basename "$d")
  steps=$(python3 -c "import sqlite3;print(max(1,sqlite3.connect('$db').execute(\"select count(*) from kernels where name like 'adamw%'\").fetchone()[0]))")
  python3 tools/profdb.py "$db" "$steps" 60 --csv "gpurun_out/${n}_stats.csv" > "gpurun_out/${n}_summary.txt" 2>&1
  python3 tools/timeline.py "$db" 5 >> "gpurun_out/${n}_summary.txt" 2>&1
  gzip -f "$db"
done
find gpurun_out -path "gpurun_out/${T}_*" -name "*.csv" -size +512k -exec gzip -f {} \;
du -sh gpurun_out
