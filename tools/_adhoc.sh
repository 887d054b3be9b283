cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ht
for v in base spin base2 spin2; do
  if [ "${v:0:4}" = spin ]; then export NBG_SPIN_SYNC=1; else unset NBG_SPIN_SYNC; fi
  NBG_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --steps 3 --sp-pairs 0 --no-cpu-baseline --no-profile > gpurun_out/ht/$v.json 2>gpurun_out/ht/$v.log || exit 1
done
