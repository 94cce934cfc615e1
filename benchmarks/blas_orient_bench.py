"""hipBLASLt orientation check for mixed-step projections (129..300 rows): y = x @ W^T (F.linear, the model's
call) vs y^T = W @ x^T (the transposed problem: the library sees a tall-skinny M' = N, N' = rows) plus the
transpose back to [rows, N]. Prints one JSON line per (shape, rows)."""
import argparse
import json

import torch
import torch.nn.functional as F

SHAPES = {"8b.qkv": (6144, 4096), "8b.o": (4096, 4096), "8b.gate_up": (28672, 4096), "8b.down": (4096, 14336)}


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="130,160,200,256,300")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in args.shapes.split(","):
        N, K = SHAPES[name]
        w = torch.randn(N, K, dtype=torch.bfloat16, device=dev) * 0.02
        for M in map(int, args.rows.split(",")):
            x = torch.randn(M, K, dtype=torch.bfloat16, device=dev)
            t_lin = timeit(lambda: F.linear(x, w))
            t_t = timeit(lambda: torch.mm(w, x.t()))
            t_tc = timeit(lambda: torch.mm(w, x.t()).t().contiguous())
            err = (F.linear(x, w).float() - torch.mm(w, x.t()).t().float()).abs().max().item()
            print(json.dumps({"shape": name, "M": M, "linear_us": round(t_lin, 1), "wxT_us": round(t_t, 1),
                              "wxT_plus_transpose_us": round(t_tc, 1), "TB/s_linear": round(N * K * 2 / t_lin / 1e6, 2),
                              "max_err": err}), flush=True)


if __name__ == "__main__":
    main()
