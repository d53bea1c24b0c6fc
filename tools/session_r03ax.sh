# round-3 session ax: the convolution's new default (48-row block tiles, stores paced at vmcnt(2)) —
# parity of every convolution test, the bench lines of configs 2 / 4 / 5, and PMC records of the
# new default instance (kernel trace + FETCH_SIZE / WRITE_SIZE passes of their own)
S=("convx_parity_r03ax|500|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'conv or gaussian or halo'")
for c in c2 c4 c5; do
  st=200; [ $c = c2 ] || st=20
  S+=("bench_conv_${c}_r03ax|300|python3 bench.py --op conv --config $c --steps $st --warmup 3 --no-cpu")
  S+=("convx_trace_${c}|300|rocprofv3 --kernel-trace --stats -d gpurun_out/convx_trace_${c} -o run --output-format csv -- python3 bench.py --op conv --config $c --steps $st --warmup 3 --no-cpu")
  S+=("convx_fetch_${c}|200|timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/convx_fetch_${c} -o run --output-format csv -- python3 bench.py --op conv --config $c --steps 3 --warmup 1 --no-cpu")
  S+=("convx_write_${c}|200|timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/convx_write_${c} -o run --output-format csv -- python3 bench.py --op conv --config $c --steps 3 --warmup 1 --no-cpu")
done
exec tools/gpu_session.sh "${S[@]}"
