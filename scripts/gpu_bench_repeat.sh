set -u
mkdir -p gpurun_out/var
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --step-times > gpurun_out/var/b$i.log 2>&1 || exit 1
  grep -h '^{"metric"' gpurun_out/var/b$i.log | cut -c100-190
done
