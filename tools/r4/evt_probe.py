"""Host cost of HIP event calls on a completed event (torch.cuda.Event wraps
hipEventRecord / hipEventSynchronize / hipEventElapsedTime / hipEventQuery)."""
import time
import torch

s = torch.cuda.Stream()
x = torch.zeros(1 << 20, device="cuda")
with torch.cuda.stream(s):
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    x.add_(1)
    b.record()
torch.cuda.synchronize()
for name, f in (("elapsed_time", lambda: a.elapsed_time(b)), ("synchronize", b.synchronize), ("query", b.query)):
    f()
    t = time.perf_counter()
    for _ in range(1000):
        f()
    print(f"{name}: {1e6 * (time.perf_counter() - t) / 1000:.2f} us per call", flush=True)
