# Exact-byte (32-B request) traffic of k_build v15 and k_conv_blk at 4096^2 (round 5): separate passes
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --variant 15 --tile-order 0 --zero-window 1 --steps 5 --warmup 1 --no-cpu"
C="$R/bench.py --op conv --steps 5 --warmup 1 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum -d $R/gpurun_out/p32_build_rd -o run --output-format csv -- python3 $B > $R/gpurun_out/p32_build_rd.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_64B_sum -d $R/gpurun_out/p32_build_wr -o run --output-format csv -- python3 $B > $R/gpurun_out/p32_build_wr.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum -d $R/gpurun_out/p32_conv_rd -o run --output-format csv -- python3 $C > $R/gpurun_out/p32_conv_rd.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_64B_sum -d $R/gpurun_out/p32_conv_wr -o run --output-format csv -- python3 $C > $R/gpurun_out/p32_conv_wr.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/p32_conv_fetch -o run --output-format csv -- python3 $C > $R/gpurun_out/p32_conv_fetch.log 2>&1
echo done
