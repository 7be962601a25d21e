"""Diagnostic: GPU-side timeline of pipelined setup + upload + render steps
(run on the GPU box).  The renderer runs on torch's current stream, so torch
events bracket the upload's copies and the render on the GPU's own clock."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ptlumi_loader

P = ptlumi_loader.load()
N = P.native
cfg = N.RenderConfig.make(1280, 720, 1024)
scene = N.Scene(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets"), cfg)
r = P.GpuRenderer(0)
stream = torch.cuda.current_stream()
r.set_stream(stream)
scene.setup_frame(0)
r.upload(scene, include_static=True)
img = torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda:0")
r.render(cfg, out_bgra=img)
torch.cuda.synchronize()
K = 5
ev = []
host = []
t0 = time.perf_counter()
for k in range(K):
    a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    h0 = time.perf_counter()
    scene.setup_frame(0)
    h1 = time.perf_counter()
    a.record(stream)
    r.upload(scene, include_static=False)
    b.record(stream)
    h2 = time.perf_counter()
    r.render(cfg, out_bgra=img)
    c.record(stream)
    h3 = time.perf_counter()
    ev.append((a, b, c))
    host.append((h1 - h0, h2 - h1, h3 - h2))
torch.cuda.synchronize()
print("wall per step %.1f ms" % ((time.perf_counter() - t0) / K * 1e3))
for k, ((a, b, c), (hs, hu, hr)) in enumerate(zip(ev, host)):
    gap = ev[k - 1][2].elapsed_time(a) if k else 0.0
    print("step %d: gpu gap before upload %.2f ms, upload %.2f ms, render %.1f ms | host setup %.1f upload %.1f render-enqueue %.1f ms"
          % (k, gap, a.elapsed_time(b), b.elapsed_time(c), hs * 1e3, hu * 1e3, hr * 1e3), flush=True)
