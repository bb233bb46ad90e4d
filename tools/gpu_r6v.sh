# Round 6: C4 determinism hunt -- run-to-run adapter-gradient digests, N runs per variant, each compared with the
# variant's first run on the box (usage: gpu_r6v.sh TAG N [ENV=V ...])
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
tag=$1; n=$2; shift 2
for kv in "$@"; do export "$kv"; done
for rep in $(seq 1 $n); do
  f=/tmp/${tag}_$rep.txt
  timeout -k 10 120 python -u tools/lora_grad_digest.py --steps 9 --arb > $f 2> gpurun_out/${tag}.err || { tail -5 gpurun_out/${tag}.err; exit 1; }
  if [ $rep = 1 ]; then echo "$tag 1 $(grep '^step' $f | awk '{print $4}' | tr '\n' ' ')"
  else python tools/digest_diff.py /tmp/${tag}_1.txt $f; rm -f $f; fi
done
