"""Expected results of the reference ring's fold at sampled element indices (test helper).

The bucket values come from synth's index-addressable generators, so any sample of a full-size bucket generated on the GPU
is re-derived on the CPU; the fold itself runs in the C restatement (oracle/), which
tests/test_oracle.py pins to the reference."""
import numpy as np

from hydra_amd import synth


def bf16_acc32_expected(O, P, n, idx, max_segment=1 << 20, gen=synth.stress_cancel_at):
    """The reference ring's fold on bf16 values widened to fp32, at element indices idx, with
    the bf16 bucket's block geometry (O.ring_plan, the C restatement of allreduce.cc:199-221 at
    E = 2): owner block q = x_q + (x_{q+1} + (... + x_{q-1})) accumulated in fp32 by the C
    restatement (orc_acc_bf16_f32: acc + (float)b), rounded once to bf16 (RNE).  gen(P, r, idx):
    rank r's fp32 values before the bf16 rounding (synth.stress_cancel_at by default: the
    values whose bf16 result still depends on the fold order)."""
    ns, sb, S = O.ring_plan(P, n, 2, max_segment)
    block = S * sb // 2  # elements per owner block
    vals = [synth.bf16_bits(gen(P, r, idx)) for r in range(P)]
    owner = np.minimum(idx // block, P - 1)
    out = np.empty(idx.size, np.uint16)
    for q in range(P):
        sel = owner == q
        if not sel.any():
            continue
        acc = synth.bf16_to_f32(vals[(q + P - 1) % P][sel]).astype(np.float32)
        for d in range(P - 2, -1, -1):
            acc = O.acc_bf16_f32(acc, vals[(q + d) % P][sel])
        out[sel] = synth.bf16_bits(acc)
    return out, vals, (ns, sb, S)


def sample_indices(n, ns, seg, count=1 << 20, seed=55):
    """>= `count` sorted element indices of an n-element bucket: every segment boundary's two
    elements either side (ns segments of `seg` elements -- so every owner block's first and last
    elements too), the bucket's ends, and `count` uniform random ones."""
    edges = np.concatenate([np.arange(ns + 1, dtype=np.int64) * seg + d for d in (-2, -1, 0, 1)])
    rnd = np.random.default_rng(seed).integers(0, n, count, dtype=np.int64)
    idx = np.unique(np.concatenate([edges, rnd, [0, 1, n - 2, n - 1]]))
    return idx[(idx >= 0) & (idx < n)]


def device_bucket(gen, P, rank, n, dev, out_dtype, chunk=16 << 20, out=None):
    """gen(P, rank, idx) over all n indices on `dev` (synth.fill_at, chunked)."""
    return synth.fill_at(gen, P, rank, n, dev, out_dtype, chunk=chunk, out=out)
