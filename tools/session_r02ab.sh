# round-2 session: PMC traffic + kernel trace of the convolution extension's block tiles on configs
# 4 and 5 (bench.py --op conv attaches it when kernel / rows / order match)
S=()
for c in c4 c5; do
  S+=("conv_trace_$c|300|rocprofv3 --kernel-trace --stats -d gpurun_out/conv_trace_$c -o run --output-format csv -- python3 bench.py --op conv --config $c --steps 20 --warmup 2 --no-cpu")
  S+=("conv_fetch_$c|200|timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/conv_fetch_$c -o run --output-format csv -- python3 bench.py --op conv --config $c --steps 3 --warmup 1 --no-cpu")
  S+=("conv_write_$c|200|timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/conv_write_$c -o run --output-format csv -- python3 bench.py --op conv --config $c --steps 3 --warmup 1 --no-cpu")
done
exec tools/gpu_session.sh "${S[@]}"
