cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rsp
for f in 0.1 1.0; do
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rsp/f$f -o kt -f csv -- python3 $R/scripts/row_scale_probe.py $f > $R/gpurun_out/rsp/f$f.log 2>&1 || exit 1
grep -h "row_scale\|inject_wave" $R/gpurun_out/rsp/f$f/kt_kernel_stats.csv | cut -c1-200
done
