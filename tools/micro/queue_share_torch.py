"""Which of torch's streams share a hardware queue (in-order) on this box?

Runs the bounded flag-poll test of ``queue_share.hip`` on torch's default
stream and on streams drawn from torch's stream pool -- the pool
``ProcessGroupNCCL`` takes its communicator streams from -- at normal and high
priority.  Two streams "collide" when a spinning kernel on one holds back a
kernel on the other: exactly what a pre-posted RCCL receive would do to the
compute stream (or to another communicator) if they shared a queue.

Usage: python tools/micro/queue_share_torch.py [GPU_MAX_HW_QUEUES]
(the value is exported before torch loads HIP; omit it to keep the environment's).
"""
import ctypes
import os
import sys

if len(sys.argv) > 1:
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[1]

import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main() -> None:
    lib = ctypes.CDLL(os.path.join(HERE, "queue_share_lib.so"))
    dev = torch.device("cuda:0")
    flag = torch.zeros(64, dtype=torch.int32, device=dev)
    out = torch.zeros(64, dtype=torch.int64, device=dev)
    default = torch.cuda.default_stream(dev)
    normal = [torch.cuda.Stream(dev) for _ in range(12)]
    high = [torch.cuda.Stream(dev, priority=-1) for _ in range(12)]
    named = [("default", default)] + [(f"pool{i}", s) for i, s in enumerate(normal)] + \
            [(f"high{i}", s) for i, s in enumerate(high)]

    def collides(a, b) -> bool:
        flag.zero_()
        torch.cuda.synchronize()
        assert lib.qs_launch_waiter(ctypes.c_void_p(a.cuda_stream), ctypes.c_void_p(flag.data_ptr()),
                                    ctypes.c_void_p(out.data_ptr())) == 0
        assert lib.qs_launch_setter(ctypes.c_void_p(b.cuda_stream), ctypes.c_void_p(flag.data_ptr())) == 0
        torch.cuda.synchronize()
        return int(out[0]) < 0

    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', '(unset)')}: "
          f"default stream + {len(normal)} normal-priority + {len(high)} high-priority pool streams")
    pairs = []
    for x in range(len(named)):
        for y in range(x + 1, len(named)):
            if collides(named[x][1], named[y][1]):
                pairs.append(f"{named[x][0]}~{named[y][0]}")
    print(f"  colliding (serialised) pairs: {len(pairs)} of {len(named) * (len(named) - 1) // 2}")
    print("  " + (", ".join(pairs) if pairs else "none"))


if __name__ == "__main__":
    main()
