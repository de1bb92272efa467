#!/usr/bin/env python3
"""Which HW queue does a HIP stream land on? (strong-scaling replay bimodality, profiles/r04/streams)

Run under `rocprofv3 --kernel-trace --output-format csv -d DIR -o q -- python tools/micro/queue_map.py`:
launches one small kernel per stream, tagged by the launch order, for (a) torch pool streams,
(b) high-priority torch pool streams, (c) streams made with hipExtStreamCreateWithCUMask (all CUs
enabled), then prints the stream handles in order; Queue_Id per dispatch comes from the trace."""
import ctypes

import torch


def main():
    dev = torch.device("cuda", 0)
    x = torch.zeros(1 << 20, device=dev)
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    out = []
    pools = {"pool": [torch.cuda.Stream(dev) for _ in range(6)],
             "pool_hi": [torch.cuda.Stream(dev, priority=-1) for _ in range(4)]}
    cm = []
    for _ in range(6):
        s = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask) == 0
        cm.append(torch.cuda.ExternalStream(s.value, device=dev))
    pools["cumask"] = cm
    for name, streams in pools.items():
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                for _ in range(3):
                    x.add_(1.0)
            torch.cuda.synchronize(dev)
            out.append((name, i, hex(s.cuda_stream)))
    for o in out:
        print(*o)


if __name__ == "__main__":
    main()
