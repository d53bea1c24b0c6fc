"""PCIe / host-copy ceilings for the host-mirror path: one 447 MB device->pinned
copy, the same on two streams and as 32 MiB chunks, and host memcpy with 1-16 threads."""
import time, torch, numpy as np, threading
n = 447 * 1024 * 1024 // 4
d = torch.empty(n, dtype=torch.float32, device="cuda").fill_(1.0)
h = torch.empty(n, dtype=torch.float32).pin_memory()
for _ in range(2):
    torch.cuda.synchronize(); t=time.perf_counter(); h.copy_(d, non_blocking=True); torch.cuda.synchronize(); dt=time.perf_counter()-t
print("D2H one copy 447MB: %.2f ms %.1f GB/s" % (dt*1e3, n*4/dt/1e9))
# two streams, two halves
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
half = n // 2
for _ in range(2):
    torch.cuda.synchronize(); t=time.perf_counter()
    with torch.cuda.stream(s1): h[:half].copy_(d[:half], non_blocking=True)
    with torch.cuda.stream(s2): h[half:].copy_(d[half:], non_blocking=True)
    torch.cuda.synchronize(); dt=time.perf_counter()-t
print("D2H two streams: %.2f ms %.1f GB/s" % (dt*1e3, n*4/dt/1e9))
# chunked 32 MiB copies on one stream
ch = 32*1024*1024//4
for _ in range(2):
    torch.cuda.synchronize(); t=time.perf_counter()
    for i in range(0, n, ch): h[i:i+ch].copy_(d[i:i+ch], non_blocking=True)
    torch.cuda.synchronize(); dt=time.perf_counter()-t
print("D2H 32MiB chunks: %.2f ms %.1f GB/s" % (dt*1e3, n*4/dt/1e9))
a = np.ones(n, dtype=np.float32); b = np.empty_like(a)
for T in (1, 4, 8, 16):
    parts = np.array_split(np.arange(n), T)
    def work(p): b[p[0]:p[-1]+1] = a[p[0]:p[-1]+1]
    t=time.perf_counter()
    th=[threading.Thread(target=work, args=(p,)) for p in parts]
    [x.start() for x in th]; [x.join() for x in th]
    dt=time.perf_counter()-t
    print("host memcpy %d threads: %.1f GB/s" % (T, n*4/dt/1e9))
