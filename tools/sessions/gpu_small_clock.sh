# tools/gpu_small_clock.sh -- GPU clock per launch (GRBM_GUI_ACTIVE cycles /
# duration) over back-to-back uniform 4 KiB launches (writes gpurun_out/sclk/)
set -o pipefail
R=$PWD
O=$R/gpurun_out/sclk
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/clk -o run -- python3 $R/tools/small_uniform.py 4096 10 > $O/clk.log 2>&1 || exit 1
