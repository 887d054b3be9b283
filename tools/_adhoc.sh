cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/var2
for v in base vt8 nostore; do
  if [ $v = base ]; then L=nebula_amd/libnbg.so; else L=build/variants/libnbg_$v.so; fi
  NBG_LIB=$L timeout -k 10 200 python -u bench.py --steps 2 --sp-pairs 0 --no-cpu-baseline > gpurun_out/var2/$v.json 2>gpurun_out/var2/$v.log || exit 1
  NBG_LIB=$L timeout -k 10 200 python -u bench.py --steps 2 --sp-pairs 0 --no-cpu-baseline --no-profile > gpurun_out/var2/${v}_np.json 2>>gpurun_out/var2/$v.log || exit 1
  echo "$v done"
done
