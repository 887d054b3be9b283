#!/bin/bash
# Same-box A/B of an SP switch (env var $2, values 0/1 alternating).  Usage: bash tools/sp_ab.sh <tag> <VAR>
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_path.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_path.log" 2>&1 \
  || { tail -20 "$OUT/pytest_path.log"; exit 1; }
echo "tests done"
for v in 0 1 0 1; do
  env "$2=$v" timeout -k 10 300 python -u bench.py --steps 1 --sp-pairs 10000 --no-cpu-baseline --no-profile --c5-scale 0 \
    > "$OUT/sp_$2_$v.$RANDOM.json" 2>> "$OUT/ab.log" || { tail -20 "$OUT/ab.log"; exit 1; }
  echo "run $v done"
done
