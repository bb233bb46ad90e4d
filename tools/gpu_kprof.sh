# Kernel durations of a micro-benchmark from rocprofv3 (host launch gaps excluded).
# usage: bash tools/gpu_kprof.sh <tag> <python script> [args]
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/kp_${TAG}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kp_${TAG} -o run -- python3 -u "$@" > gpurun_out/kp_${TAG}.log 2>&1 || { echo "kprof failed"; tail -20 gpurun_out/kp_${TAG}.log; exit 1; }
DB=$(find gpurun_out/kp_${TAG} -name '*.db' | head -1)
python3 -c "
import sqlite3
c = sqlite3.connect('$DB')
rows = c.execute('select name, count(*), sum(end - start), avg(end - start) from kernels group by name order by sum(end - start) desc').fetchall()
for n, k, tot, avg in rows[:30]:
    print(f'{avg / 1e3:9.2f} us x{k:5d}  {n[:110]}')
"
rm -rf gpurun_out/kp_${TAG}
