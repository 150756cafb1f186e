#!/usr/bin/env python3
"""RCCL rehearsal of bench.py's N > 1 collectives on a one-GPU box: a world-1
"nccl" process group (RCCL) on cuda:0 runs exactly the calls the multi-GPU
bench makes -- dist.gather of a complex tensor moved as real pairs (the result
gather), a float64 MAX all-reduce (max over ranks of the wall time), an int64
MIN all-reduce (the correlator's first detection) and barriers -- through the
srcdsp_amd.dist helpers with their world == 1 shortcuts bypassed.  Prints one
JSON line; exit 1 on any mismatch.  (Two ranks cannot share one GPU under
RCCL; the driver's multi-GPU node runs N > 1.)"""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from srcdsp_amd import dist as D  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ok = {}
    y = torch.randn(8, 4096, dtype=torch.complex64, device="cuda")
    src = torch.view_as_real(y)
    bufs = [torch.empty_like(src)]
    dist.gather(src, bufs, dst=0)
    ok["gather"] = bool(torch.equal(torch.view_as_complex(bufs[0]), y))
    t = torch.tensor([1.25], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok["max_f64"] = float(t.item()) == 1.25
    t = torch.tensor([D.NO_DETECTION - 5], dtype=torch.int64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    ok["min_i64"] = int(t.item()) == D.NO_DETECTION - 5
    dist.barrier()
    torch.cuda.synchronize()
    ok["backend"] = dist.get_backend()
    ok["world"] = dist.get_world_size()
    dist.destroy_process_group()
    print(json.dumps(ok), flush=True)
    sys.exit(0 if all(v for k, v in ok.items() if isinstance(v, bool)) else 1)


if __name__ == "__main__":
    main()
