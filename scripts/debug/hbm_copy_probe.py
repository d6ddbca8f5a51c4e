"""What a plain device copy reaches on this box (the roofline the memory-bound LayerNorm passes
are judged against): torch copy_ and hipMemcpyAsync (D2D) of 1.5 GB, read + write bytes / time."""
import json
import torch


def main():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for nbytes in (512 << 20, 1536 << 20, 3 << 30):
        a = torch.empty(nbytes // 4, device="cuda", dtype=torch.float32).normal_()
        b = torch.empty_like(a)
        for name, fn in (("torch_copy", lambda: b.copy_(a)), ("add_inplace_rw", lambda: a.add_(1.0))):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(10):
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            t = ts[len(ts) // 2] * 1e-3
            print(json.dumps({"op": name, "MB": nbytes >> 20, "ms": round(t * 1e3, 3),
                              "TBps_read_plus_write": round(2 * nbytes / t / 1e12, 2)}), flush=True)
        del a, b


if __name__ == "__main__":
    main()
