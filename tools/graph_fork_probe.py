"""Does a captured HIP graph run two independent branches concurrently on this ROCm?  Captures
sleep(X) on the capture stream ‖ sleep(X) on a forked side stream, joined, and compares the replay time
with a graph of the two sleeps in sequence (a diagnostic for the scan-beside-fixup layout)."""
import time

import torch


def main():
    cyc = 2_000_000
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    gp, gs = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(s1):
        with torch.cuda.graph(gp, stream=s1):
            s2.wait_stream(s1)
            torch.cuda._sleep(cyc)
            with torch.cuda.stream(s2):
                torch.cuda._sleep(cyc)
            s1.wait_stream(s2)
        with torch.cuda.graph(gs, stream=s1):
            torch.cuda._sleep(cyc)
            torch.cuda._sleep(cyc)
    for name, g in (("parallel", gp), ("serial", gs), ("parallel", gp), ("serial", gs)):
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        print(f"{name}: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us/replay", flush=True)
    # eager two streams for comparison
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        s2.wait_stream(s1)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cyc)
        s1.wait_stream(s2)
    torch.cuda.synchronize()
    print(f"eager two streams: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us/iter", flush=True)


if __name__ == "__main__":
    main()
