set -u
cd "${GRAFT_REPO_ROOT}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
O=gpurun_out/pmc_stencil; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "diffuse_stencil" -d $O/fetch -o run --output-format csv -- python scripts/diffuse_bench.py --dtypes bf16 fp32 --iters 3 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "diffuse_stencil" -d $O/write -o run --output-format csv -- python scripts/diffuse_bench.py --dtypes bf16 fp32 --iters 3 > $O/write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "diffuse_stencil" -d $O/trace -o run --output-format csv -- python scripts/diffuse_bench.py --dtypes bf16 fp32 --iters 10 > $O/trace.log 2>&1 || exit $?
