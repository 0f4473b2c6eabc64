set -e
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 > "$ROOT/gpurun_out/prof_bench.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex 'kl::' --output-format csv -d "$ROOT/gpurun_out/pmcF" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-p2m --steps 5 --warmup 2 > "$ROOT/gpurun_out/pmcF.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex 'kl::' --output-format csv -d "$ROOT/gpurun_out/pmcW" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-p2m --steps 5 --warmup 2 > "$ROOT/gpurun_out/pmcW.log" 2>&1
