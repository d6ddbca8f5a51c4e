"""Generation throughput: nanoGPT's recompute loop vs KV-cache decoding (eager / HIP graph).

Random-init GPT-2 weights of the named size, bf16, a random prompt of --prompt tokens,
--new tokens sampled per sequence (temperature 0.8, top-k 200 as in sample.py).  Prints
one JSON line per (model, batch, mode) with new tokens/s over the whole batch and the
per-token latency.

    python scripts/decode_bench.py [--models gpt2,gpt2-xl] [--batches 1,8,64] [--prompt 128] [--new 256]
"""

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.models import GPT, GPTConfig  # noqa: E402
from nanosandbox_amd.runtime.decode import Decoder  # noqa: E402

DIMS = {"gpt2": (12, 12, 768), "gpt2-medium": (24, 16, 1024), "gpt2-large": (36, 20, 1280), "gpt2-xl": (48, 25, 1600)}


def run_cached(model, idx, new, use_graph):
    B = idx.shape[0]
    dec = Decoder(model, B, use_graph=use_graph)
    dec.sample_into(dec.prefill(idx), 0.8, 200)
    if use_graph:
        dec.run(1, 0.8, 200)  # capture outside the timed loop
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if use_graph:
        dec.run(new, 0.8, 200)  # step + sampling + feedback: one graph replay per token
    else:
        for _ in range(new):  # eager step + the same device sampling kernel
            dec.sample_into(dec.step(dec.tok), 0.8, 200)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dec.release()
    return dt


def run_recompute(model, idx, new):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.generate(idx, new, temperature=0.8, top_k=200)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="gpt2,gpt2-xl")
    ap.add_argument("--batches", default="1,8,64")
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--recompute-new", type=int, default=32, help="tokens timed for the recompute loop (slow)")
    ap.add_argument("--modes", default="recompute,cached,graph")
    a = ap.parse_args()
    for name in a.models.split(","):
        L, H, C = DIMS[name]
        torch.manual_seed(0)
        model = GPT(GPTConfig(n_layer=L, n_head=H, n_embd=C, dropout=0.0, bias=True)).eval().cuda()
        model.set_compute_dtype(torch.bfloat16)
        for B in [int(b) for b in a.batches.split(",")]:
            idx = torch.randint(0, 50257, (B, a.prompt), device="cuda")
            with torch.no_grad():
                for mode in a.modes.split(","):
                    if mode == "recompute":
                        run_recompute(model, idx, 2)  # warm-up (tuner, allocator)
                        n = a.recompute_new
                        dt = run_recompute(model, idx, n)
                    else:
                        n = a.new
                        run_cached(model, idx, 4, mode == "graph")
                        dt = run_cached(model, idx, n, mode == "graph")
                    print(json.dumps({"model": name, "batch": B, "mode": mode, "prompt": a.prompt, "new_tokens": n,
                                      "tokens_per_s": round(B * n / dt, 1), "ms_per_token": round(dt / n * 1e3, 3)}),
                          flush=True)
        del model
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
