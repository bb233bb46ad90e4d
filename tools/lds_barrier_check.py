"""Static check of gfx950 device assembly (not a test by itself; tests/test_lds_barriers.py runs it on attention.hip):
every s_barrier must be reached with no LDS access of this wave outstanding.

Why: gfx950's s_barrier does not wait for a wave's outstanding ds_reads or ds_writes.  The ring kernels refill the
slot read in the previous tile with LDS-DMA right after the barrier, so a wave that arrives with ds_reads still in
flight lets another wave's DMA overwrite the data under them.  The compiler creates exactly that when it sinks the
last MFMA of a tile -- and the lgkmcnt wait for its operands -- below a raw s_barrier (attn_bwd_dq_kernel<64, 3>
before round 6: dQ differed run to run when co-resident kernels slowed its LDS reads).

A forward data flow over each kernel's basic blocks: an LDS access counts as outstanding until an lgkmcnt wait that
covers it (a write published to other waves by the barrier is a RAW hazard just as a read is a WAR one), and a block starts with the most reads outstanding over its predecessors.

usage: python tools/lds_barrier_check.py FILE.hip|FILE.s ...   (exit 1 on a hit)
"""
import os
import re
import subprocess
import sys
import tempfile

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "onetrainer_amd", "csrc")


def device_asm(src: str) -> str:
    if src.endswith(".s"):
        return open(src).read()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", CSRC,
                        "--cuda-device-only", "-S", "-o", out, src], check=True, capture_output=True)
        return open(out).read()


def _blocks(body):
    """basic blocks of one kernel: [(label, [instructions], [successor labels])]"""
    blocks, cur, label = [], [], "entry"
    for raw in body:
        m = re.match(r"^(\.LBB\w+):", raw)
        if m:
            blocks.append([label, cur])
            label, cur = m.group(1), []
            continue
        ins = raw.strip()
        if ins and not ins.startswith(";") and not ins.startswith("."):
            cur.append(ins)
    blocks.append([label, cur])
    out = []
    for i, (lab, ins) in enumerate(blocks):
        succ, falls = [], True
        for t in ins:
            b = re.match(r"s_(c?)branch\w*\s+(\.LBB\w+)", t)
            if b:
                succ.append(b.group(2))
                if not b.group(1):
                    falls = False
            if t.startswith("s_endpgm"):
                falls = False
        if falls and i + 1 < len(blocks):
            succ.append(blocks[i + 1][0])
        out.append((lab, ins, succ))
    return out


def _transfer(ins, pending):
    """-> (pending after the block, barriers, barriers reached with reads outstanding)"""
    nb = bad = 0
    for t in ins:
        if t.startswith("ds_") and not t.startswith("ds_nop") and not t.startswith("ds_swizzle") \
                and not t.startswith("ds_bpermute") and not t.startswith("ds_permute"):
            pending = min(pending + 1, 64)   # LDS reads, writes and atomics (lane permutes touch no LDS)
        w = re.search(r"s_waitcnt.*lgkmcnt\((\d+)\)", t)
        if w:
            n = int(w.group(1))
            pending = 0 if n == 0 else min(pending, n)
        if t.startswith("s_barrier"):
            nb += 1
            bad += pending > 0
    return pending, nb, bad


def scan(asm: str):
    """-> [(kernel, barriers, barriers reached with LDS reads possibly outstanding)]: a forward data flow over each
    kernel's basic blocks (outstanding reads at a block entry = the most over its predecessors)"""
    lines = asm.split("\n")
    out, name, body = [], None, []
    for raw in lines:
        m = re.match(r"^(_Z\w+):", raw)
        if m:
            name, body = m.group(1), []
            continue
        if name is None:
            continue
        if raw.startswith(".Lfunc_end"):
            blocks = _blocks(body)
            idx = {lab: i for i, (lab, _, _) in enumerate(blocks)}
            pin = [0] * len(blocks)
            changed = True
            while changed:
                changed = False
                for i, (_, ins, succ) in enumerate(blocks):
                    po, _, _ = _transfer(ins, pin[i])
                    for s_ in succ:
                        j = idx.get(s_)
                        if j is not None and po > pin[j]:
                            pin[j] = po
                            changed = True
            nb = bad = 0
            for i, (_, ins, _) in enumerate(blocks):
                _, b1, b2 = _transfer(ins, pin[i])
                nb += b1
                bad += b2
            out.append((name, nb, bad))
            name = None
            continue
        body.append(raw)
    return out


def main():
    hits = 0
    for src in sys.argv[1:]:
        for name, nb, bad in scan(device_asm(src)):
            if bad:
                hits += 1
                print(f"{os.path.basename(src)}: {name}: {bad} of {nb} barriers with LDS reads outstanding")
    print("LDS-barrier hits:", hits)
    return 1 if hits else 0


if __name__ == "__main__":
    sys.exit(main())
