"""Does a captured HIP graph keep two-stream concurrency on this ROCm?  Times K
independent matmul chains on 1 stream vs 2 streams, eager and graph-replayed.
    python tools/graph_concurrency.py"""
import time
import torch

dev = "cuda"
a = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
b = [torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16) for _ in range(2)]
# small matmuls (under-fill the chip) so that two streams can overlap
xs = [torch.randn(256, 2048, device=dev, dtype=torch.bfloat16) for _ in range(2)]
s1 = torch.cuda.Stream()
N = 50


def work(two):
    main = torch.cuda.current_stream()
    if two:
        s1.wait_stream(main)
        with torch.cuda.stream(s1):
            y = xs[1]
            for _ in range(N):
                y = torch.mm(y, b[1])
        x = xs[0]
        for _ in range(N):
            x = torch.mm(x, b[0])
        main.wait_stream(s1)
    else:
        x, y = xs[0], xs[1]
        for _ in range(N):
            x = torch.mm(x, b[0])
        for _ in range(N):
            y = torch.mm(y, b[1])


def bench(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for two in (False, True):
    e = bench(lambda: work(two))
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        work(two)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            work(two)
    torch.cuda.current_stream().wait_stream(s)
    r = bench(g.replay)
    print(f"{'2 streams' if two else '1 stream '}: eager {e:.3f} ms  graph {r:.3f} ms", flush=True)
