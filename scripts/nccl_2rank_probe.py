"""Probe (tuning/rehearsal only): can two ranks on ONE GPU form an RCCL process
group?  Run under torch.distributed.run --nproc-per-node 2."""
import os
import torch
import torch.distributed as dist

local = int(os.environ["LOCAL_RANK"])
torch.cuda.set_device(local % torch.cuda.device_count())
dist.init_process_group("nccl", device_id=torch.device("cuda", local % torch.cuda.device_count()))
t = torch.ones(4, device="cuda") * (dist.get_rank() + 1)
dist.all_reduce(t)
print(f"rank {dist.get_rank()} all_reduce -> {t.tolist()}", flush=True)
dist.destroy_process_group()
