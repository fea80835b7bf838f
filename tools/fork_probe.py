"""Cost of cross-stream fork / join edges inside a captured HIP graph (diagnostic; not a test).

Each variant is a chain of spin kernels (torch.cuda._sleep) captured into one graph and replayed; the replay time
against the chain without side branches is the edges' cost.
    python tools/fork_probe.py"""
import torch

CYC = 20000


def timed(fn, reps=200):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.synchronize()
    for _ in range(10):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


side = None


def chain(n):
    for _ in range(n):
        torch.cuda._sleep(CYC)


def fork_join(k_before, k_side, k_main, k_after, early=0):
    """main: k_before spins, fork (side waits on the main stream, or on an event `early` spins back), side: k_side
    spins, main: k_main spins, join, main: k_after spins."""
    global side
    cur = torch.cuda.current_stream()
    ev = None
    for i in range(k_before):
        if early and i == k_before - early:
            ev = torch.cuda.Event()
            ev.record(cur)
        torch.cuda._sleep(CYC)
    if ev is None:
        side.wait_stream(cur)
    else:
        side.wait_event(ev)
    with torch.cuda.stream(side):
        for _ in range(k_side):
            torch.cuda._sleep(CYC)
    for _ in range(k_main):
        torch.cuda._sleep(CYC)
    cur.wait_stream(side)
    for _ in range(k_after):
        torch.cuda._sleep(CYC)


def main():
    global side
    side = torch.cuda.Stream()
    base = timed(lambda: chain(6))
    print(f"chain of 6 spins: {base:.1f} us ({base / 6:.2f} per spin)")
    one = base / 6
    v = timed(lambda: fork_join(3, 1, 1, 1))
    print(f"3 | fork: side 1 || main 1 | join | 1   : {v:.1f} us  (edges cost {v - 5 * one:.1f} us over 5 serial spins)")
    v = timed(lambda: fork_join(3, 1, 0, 1))
    print(f"3 | fork: side 1 | join | 1 (no main work) : {v:.1f} us  (edges cost {v - 5 * one:.1f})")
    v = timed(lambda: fork_join(3, 0, 1, 1))
    print(f"3 | fork: side 0 || main 1 | join | 1   : {v:.1f} us  (edges cost {v - 5 * one:.1f})")
    v = timed(lambda: fork_join(3, 1, 1, 1, early=2))
    print(f"fork 2 spins early, side 1 || main 1    : {v:.1f} us  (edges cost {v - 5 * one:.1f})")
    v = timed(lambda: fork_join(3, 1, 2, 1, early=2))
    print(f"fork 2 spins early, side 1 || main 2    : {v:.1f} us  (vs 6 serial: {v - 6 * one:.1f})")
    for k in (2, 4):
        v = timed(lambda: fork_join(1, k, k, 1))
        print(f"1 | fork: side {k} || main {k} | join | 1 : {v:.1f} us  (ideal {(2 + k) * one:.1f}, serial "
              f"{(2 + 2 * k) * one:.1f})")
    v = timed(lambda: fork_join(1, 2, 0, 3))
    print(f"1 | fork: side 2 | join | 3 (main idle) : {v:.1f} us  (serial {6 * one:.1f})")


if __name__ == "__main__":
    main()
