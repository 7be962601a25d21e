"""Diagnostic: where the per-frame setup + upload time goes (run on the GPU box).
Times K steps of: render only; upload + render; setup + upload + render."""
import sys
import os
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ptlumi_loader

P = ptlumi_loader.load()
N = P.native
cfg = N.RenderConfig.make(1280, 720, int(sys.argv[1]) if len(sys.argv) > 1 else 1024)
scene = N.Scene(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets"), cfg)
r = P.GpuRenderer(0)
scene.setup_frame(0)
r.upload(scene, include_static=True)
img = torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda:0")
K = 4


def run(name, fn):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    host = []
    for _ in range(K):
        h0 = time.perf_counter()
        fn()
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / K
    print("%-26s %8.1f ms/step   host %s ms" % (name, el * 1e3, [round(x * 1e3, 1) for x in host]), flush=True)


run("render", lambda: r.render(cfg, out_bgra=img))
run("upload+render", lambda: (r.upload(scene, include_static=False), r.render(cfg, out_bgra=img)))
run("setup+upload+render", lambda: (scene.setup_frame(0), r.upload(scene, include_static=False), r.render(cfg, out_bgra=img)))
t = time.perf_counter()
for _ in range(K):
    r.upload(scene, include_static=False)
torch.cuda.synchronize()
print("upload alone %.1f ms" % ((time.perf_counter() - t) / K * 1e3))


def timed_sync(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


for _ in range(2):
    a = timed_sync(lambda: r.render(cfg, out_bgra=img))
    b = timed_sync(lambda: r.render(cfg, out_bgra=img))
    u = timed_sync(lambda: r.upload(scene, include_static=False))
    c = timed_sync(lambda: r.render(cfg, out_bgra=img))
    print("render %.1f, render %.1f, upload (synced) %.1f, render after upload %.1f ms" % (a, b, u, c), flush=True)
host = torch.empty(51 << 20, dtype=torch.uint8, pin_memory=True)
devb = torch.empty(51 << 20, dtype=torch.uint8, device="cuda:0")
for _ in range(3):
    print("51 MB pinned H2D %.2f ms" % timed_sync(lambda: devb.copy_(host, non_blocking=True)), flush=True)
