"""Publication times of the pictures of one pipelined run (HL_AMD_TRACE_WRITERS):
the first picture's latency and the steady lag between pictures.
  python tools/base_run_trace.py W H N [workgroups [reach]]"""
import os
import sys

os.environ["HL_AMD_TRACE_WRITERS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hartallo_amd import _lib  # noqa: E402

if os.environ.get("HL_LIB"):
    _lib.load_library(os.environ["HL_LIB"])
from hartallo_amd import Encoder, synth  # noqa: E402

W, H, N = (int(v) for v in sys.argv[1:4])
wg = int(sys.argv[4]) if len(sys.argv) > 4 else 0
reach = int(sys.argv[5]) if len(sys.argv) > 5 else 2
clip = synth.clip(W, H, N, 41)
dev = torch.from_numpy(clip).cuda()
ny, nc = W * H, W * H // 4
ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + nc) for i in range(N)]
enc = Encoder(W, H, 28, 16, 1, 30)
if wg or reach != 2:
    enc.set_pipeline(wg, reach, 64)
enc.set_timing(True)
enc.encode_batch_device(ptrs)  # warm
enc.close()
enc = Encoder(W, H, 28, 16, 1, 30)
if wg or reach != 2:
    enc.set_pipeline(wg, reach, 64)
enc.set_timing(True)
enc.encode_batch_device(ptrs)
print(f"{W}x{H} reach {reach} workgroups {wg} kernel ms {enc.timing_ms()[1]:.1f} per picture {enc.timing_ms()[1] / N:.2f} "
      f"chain walks {enc.last_chain_walks()} reruns {enc.last_reruns()}", flush=True)
enc.close()
