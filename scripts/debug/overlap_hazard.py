"""Probe: persistent GEMMs of the backward vs a bucket all-reduce on a side stream (VERDICT r5
weak item 4 / next-round item 2), on ONE GPU.

The flat reducer (nanosandbox_amd/parallel/reducer.py) launches each gradient bucket's
all-reduce from a backward hook; RCCL runs it as a kernel of one workgroup per channel on its
own (high-priority) stream.  Our forward / input-gradient GEMMs are persistent: grid = #CUs,
one 4-wave workgroup per CU that owns the whole register file and most of the LDS, tiles
walked in a fixed per-workgroup order.  Either the collective's workgroups wait for a whole
GEMM to drain, or they take CUs a GEMM workgroup then waits for -- and with static tiles that
workgroup's whole tile chain runs late.

This probe reproduces the footprint without a second GPU: the real reducer (gloo, world 1)
with its launch replaced by ``nsa_probe_spin`` -- NWG workgroups of 256 threads, 8 KiB LDS,
each spinning SPIN_US on the real-time counter -- on a high-priority side stream that waits
for the compute stream at the hook, exactly as ProcessGroupNCCL does.  A marker kernel on the
compute stream stamps the moment the backward reached the hook.  Per NWG it reports:
  * the backward's stretch (median over reps, interleaved with no-interferer reps) against
    the CU share the interferer took (launched buckets x NWG x SPIN_US / #CUs);
  * the interferer's start delay: first / last workgroup start minus the marker.
One micro-step of the per-rank shape at N = 8 (60 x 1024 tokens), GPT-2 124M, bf16.

    python scripts/debug/overlap_hazard.py [--nwg 16,32,64] [--spin-us 400] [--reps 6]
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


class _Work:
    """What reducer.finish() waits on: the compute stream waits for the side stream."""

    def __init__(self, side):
        self.ev = torch.cuda.Event()
        self.ev.record(side)

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nwg", default="16,32,64")
    ap.add_argument("--spin-us", type=float, default=400.0)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--micro-batch", type=int, default=60)
    ap.add_argument("--bucket-mb", type=int, default=64)
    ap.add_argument("--grid-mult", type=int, default=1,
                    help="persistent NT GEMM grid = this x #CUs (ops/gemm.py NT_GRID_MULT)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("gloo", rank=0, world_size=1)
    from nanosandbox_amd.models import GPT, GPTConfig
    from nanosandbox_amd.ops import _lib
    from nanosandbox_amd.ops import gemm as G
    from nanosandbox_amd.optim import FlatParamStore
    from nanosandbox_amd.parallel import FlatBucketReducer

    G.NT_GRID_MULT = a.grid_mult
    dev = "cuda:0"
    torch.manual_seed(0)
    cfg = GPTConfig(block_size=1024, vocab_size=50304, n_layer=12, n_head=12, n_embd=768, dropout=0.0, bias=False)
    model = GPT(cfg).to(dev)
    model.set_compute_dtype(torch.bfloat16, torch.float32)  # bench.py: fp32 residual stream
    store = FlatParamStore(model, dev, compute_dtype=torch.bfloat16)
    red = FlatBucketReducer(store, bucket_cap_mb=a.bucket_mb)
    cus = G.num_cus()
    side = torch.cuda.Stream(priority=-1)  # high priority, as TORCH_NCCL_HIGH_PRIORITY=1
    nb = len(red.buckets)
    marks = torch.zeros(nb, dtype=torch.int64, device=dev)
    max_wg = max(int(v) for v in a.nwg.split(","))
    stamps = torch.zeros(nb, 2 * max_wg, dtype=torch.int64, device=dev)
    ticks = int(a.spin_us * 100)  # 100 MHz real-time counter
    state = {"nwg": 0}

    def launch(b):
        _lib.call("nsa_probe_mark", _lib.ptr(marks[b.index:b.index + 1]), _lib.stream())
        if state["nwg"] > 0:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                _lib.call("nsa_probe_spin", state["nwg"], ticks, _lib.ptr(stamps[b.index]), _lib.stream())
        b.work = _Work(side)
        b.comm_buf = store.grad[b.start:b.end]

    red._launch = launch
    idx = torch.randint(0, 50304, (a.micro_batch, 1024), device=dev)
    tgt = torch.randint(0, 50304, (a.micro_batch, 1024), device=dev)

    def micro(nwg):
        state["nwg"] = nwg
        e0, eb, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        red.prepare(True)
        e0.record()
        _, loss = model(idx, tgt)
        loss.backward()
        eb.record()
        red.finish()
        e1.record()
        store.zero_grad()
        torch.cuda.synchronize()
        early = red.launched_in_backward[-1] if red.launched_in_backward else 0
        res = {"bwd_ms": e0.elapsed_time(eb), "step_ms": e0.elapsed_time(e1), "early": early}
        if nwg > 0:
            m = marks.cpu().tolist()
            st = stamps.cpu().tolist()
            d_first, d_last = [], []
            for b in range(nb):
                starts = [st[b][2 * w] for w in range(nwg)]
                d_first.append((min(starts) - m[b]) / 100.0)
                d_last.append((max(starts) - m[b]) / 100.0)
            res["delay_first_us"] = d_first
            res["delay_last_us"] = d_last
        return res

    for _ in range(2):  # warm-up: discovery step + one launching step
        micro(0)
    configs = [0] + [int(v) for v in a.nwg.split(",")]
    runs = {c: [] for c in configs}
    for _ in range(a.reps):
        for c in configs:
            runs[c].append(micro(c))
    base = statistics.median(r["bwd_ms"] for r in runs[0])
    out = {"cus": cus, "buckets": nb, "spin_us": a.spin_us, "micro_batch": a.micro_batch, "grid_mult": a.grid_mult,
           "bwd_ms_no_interferer": round(base, 3), "rows": []}
    print(f"grid x{a.grid_mult}: backward (fwd + bwd) without interferer: {base:.3f} ms; {nb} buckets, {cus} CUs",
          flush=True)
    for c in configs[1:]:
        rs = runs[c]
        bwd = statistics.median(r["bwd_ms"] for r in rs)
        early = rs[-1]["early"]
        share = early * c * a.spin_us / 1000.0 / cus  # ms of whole-chip time the interferer took
        # buckets launched during the backward: the tail (embeddings) is launched in finish()
        dfirst = [statistics.median(r["delay_first_us"][b] for r in rs) for b in range(nb)]
        dlast = [statistics.median(r["delay_last_us"][b] for r in rs) for b in range(nb)]
        row = {"nwg": c, "bwd_ms": round(bwd, 3), "stretch_ms": round(bwd - base, 3),
               "cu_share_ms": round(share, 3), "stretch_over_share": round((bwd - base) / share, 2) if share else None,
               "buckets_in_bwd": early, "start_delay_first_us": [round(v, 1) for v in dfirst],
               "start_delay_last_us": [round(v, 1) for v in dlast]}
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
