"""Host cost of the small torch operations on Iter0's critical path (farmer 100k
shapes): mean wall time per call over repeated calls, each followed by a sync."""
import time

import torch

S, n, N = 100000, 12, 3
dev = torch.device("cuda", 0)
x = torch.randn(n * S, dtype=torch.float64, device=dev)
cols = torch.tensor([1, 2, 0], dtype=torch.int64, device=dev)
out = torch.empty((N, S), dtype=torch.float64, device=dev)
buf = torch.randn(8, dtype=torch.float64, device=dev)
pin = torch.empty(64, dtype=torch.float64, pin_memory=True)
st = torch.cuda.current_stream(dev)


def t(name, f, reps=200):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print("%-40s %8.1f us" % (name, dt * 1e6), flush=True)


t("index_select(out=) + sync", lambda: (torch.index_select(x.view(-1, S), 0, cols, out=out), st.synchronize()))
t("index_select(out=) no sync", lambda: torch.index_select(x.view(-1, S), 0, cols, out=out))
t("3 narrow copy_ no sync", lambda: [out[k].copy_(x.view(-1, S)[c]) for k, c in enumerate((1, 2, 0))])
t(".cpu() of 3 doubles", lambda: buf[:3].cpu().numpy())


def pinned():
    pin[:3].copy_(buf[:3], non_blocking=True)
    st.synchronize()
    return pin[:3].numpy().copy()


t("pinned copy + stream sync", pinned)
t("current_stream().cuda_stream", lambda: torch.cuda.current_stream(dev).cuda_stream)

# the same reads right after a large write (dirty caches, as after Iter0's solve)
big = torch.empty(25_000_000, dtype=torch.float64, device=dev)


def after_big(f):
    def g():
        big.fill_(1.0)
        st.synchronize()
        t0 = time.perf_counter()
        big[:3].add_(1.0)                     # a tiny kernel behind it (k_expect's place)
        f()
        return time.perf_counter() - t0
    return g


for name, f in (("pageable .cpu()", lambda: buf[:3].cpu().numpy()), ("pinned copy + sync", pinned),
                ("stream sync only", lambda: st.synchronize())):
    g = after_big(f)
    g()
    ts = [g() for _ in range(20)]
    print("after 200 MB write: %-28s %8.1f us" % (name, 1e6 * sum(ts) / len(ts)), flush=True)
