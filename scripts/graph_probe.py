import sys, time, os, ctypes
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/dstd-gcn_amd")
import torch, bench, dstd_native as native
dev = torch.device("cuda", 0)
model, opts, _ = bench.load_model("h36m", dev)
T = 35; x = bench.synth_input(256, T, 22, 10, 1).to(dev); y = torch.empty_like(x)
L = native.lib()
with torch.no_grad():
    for _ in range(3): model(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50): model(x)
    torch.cuda.synchronize(); te = (time.perf_counter() - t0) / 50
    yr = model(x).clone()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        model(x)
    torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
    with torch.cuda.graph(g):
        yg = model(x)
    g.replay(); torch.cuda.synchronize()
    print("graph output equal:", torch.equal(yg, yr))
    t0 = time.perf_counter()
    for _ in range(50): g.replay()
    torch.cuda.synchronize(); tg = (time.perf_counter() - t0) / 50
    print(f"eager {te*1e3:.4f} ms  graph {tg*1e3:.4f} ms")
    # events inside capture
    prof = bench.Profiler(L, 64, 1 << native.KIND_SPATIAL)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        bench.forward_profiled(model, x, y, prof)
    for _ in range(3): g2.replay()
    torch.cuda.synchronize()
    try:
        el = prof.elapsed()
        print("events in graph:", len(el), [round(m, 4) for _, _, m in el[:6]])
    except Exception as e:
        print("event timing in graph failed:", e)
