set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_vae_gpu.py > gpurun_out/r4e_tests.log 2>&1 || { tail -40 gpurun_out/r4e_tests.log; exit 1; }
tail -3 gpurun_out/r4e_tests.log
rm -rf gpurun_out/prof_r4e
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/prof_r4e -o run -- python3 -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_r4e.log 2>&1 || { tail -30 gpurun_out/prof_r4e.log; exit 1; }
DB=$(find gpurun_out/prof_r4e -name '*.db' | head -1)
python3 tools/gap_causes.py "$DB" --top 30 > gpurun_out/r4e_gaps.txt 2>&1; cat gpurun_out/r4e_gaps.txt
python3 - "$DB" <<'PY' > gpurun_out/r4e_schema.txt 2>&1
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
for (n,) in c.execute("select name from sqlite_master where type in ('view','table') order by name"):
    cols = [r[1] for r in c.execute(f"pragma table_info('{n}')")]
    print(n, cols)
PY
head -60 gpurun_out/r4e_schema.txt
rm -rf gpurun_out/prof_r4e
