"""Cross-stream event hop cost on the GPU (diagnostics): a chain of small kernels on one stream vs the
same chain with every other kernel on a second stream joined by events (torch streams = HIP
streams).   python scripts/probe_stream_hop.py"""
import json
import torch


def main():
    dev = torch.device("cuda", 0)
    x = torch.zeros(1 << 20, device=dev)
    s0 = torch.cuda.current_stream(dev)
    s1 = torch.cuda.Stream(device=dev)
    n = 200

    def same():
        for _ in range(n):
            x.add_(1.0)
            x.add_(1.0)

    def hop():
        for _ in range(n):
            x.add_(1.0)
            s1.wait_stream(s0)
            with torch.cuda.stream(s1):
                x.add_(1.0)
            s0.wait_stream(s1)

    res = {}
    for name, fn in (("same_stream", same), ("hop", hop), ("same_stream2", same), ("hop2", hop)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) * 1e3 / n
    res["hop_pair_cost_us"] = (res["hop"] + res["hop2"] - res["same_stream"] - res["same_stream2"]) / 2
    print(json.dumps(res))


if __name__ == "__main__":
    main()
