import torch, time
dev = torch.device('cuda', 0)
for mb in (32, 64, 128, 192, 256, 512, 2048, 8192):
    n = mb * 1024 * 1024 // 4
    x = torch.ones(n, dtype=torch.float32, device=dev)
    for _ in range(3): x.sum()
    torch.cuda.synchronize()
    reps = max(5, int(20000 / mb))
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): x.sum()
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"{mb:6d} MB  {ms*1e3:9.1f} us  {mb*1.048576e6/ms/1e9:8.1f} GB/s", flush=True)
    del x
