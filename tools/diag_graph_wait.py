"""Does a hipGraph replayed on stream S honour (a) an event wait S.wait_stream(C) on work still running on C and
(b) a copy enqueued on S right before the replay?  Z is produced at the end of a long queue on C; the graph on S
reads a static input filled by a copy from Z and writes W = 2 * input."""
import torch

dev = torch.device("cuda")
C = torch.cuda.current_stream()
S = torch.cuda.Stream()
n = 1 << 22
static_in = torch.zeros(n, device=dev)
g = torch.cuda.CUDAGraph()
cap = torch.cuda.Stream()
cap.wait_stream(C)
with torch.cuda.graph(g, stream=cap):
    W = static_in * 2.0
C.wait_stream(cap)
torch.cuda.synchronize()
big = torch.randn(8192, 8192, device=dev)
bad = 0
for it in range(20):
    Z = torch.empty(n, device=dev)
    for _ in range(6):  # ~ms of queued work on C before Z is written
        big @ big
    Z.fill_(float(it + 1))
    S.wait_stream(C)
    with torch.cuda.stream(S):
        static_in.copy_(Z)
        g.replay()
        out = W.clone()
    C.wait_stream(S)
    torch.cuda.synchronize()
    ok = bool(torch.all(out == 2.0 * (it + 1)))
    bad += not ok
    if not ok:
        print("iteration", it, "stale values seen:", torch.unique(out)[:8].tolist(), flush=True)
print("stale replays:", bad, "of 20", flush=True)
