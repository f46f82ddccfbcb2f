import os, torch, torch.distributed as dist
r = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((1 << 20,), float(r + 1), device="cuda")
dist.reduce(t, 0)
torch.cuda.synchronize()
print("rank", r, "ok", t[0].item(), flush=True)
dist.destroy_process_group()
