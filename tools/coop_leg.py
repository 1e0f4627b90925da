"""The bench's 4096-bus diagnostic leg alone (the paired wave-block kernel
beside the exact generic kernel): tools/runs/gpu_r03aa.sh times it."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
stream = torch.cuda.current_stream(dev)
print(json.dumps(bench._diag_4096(torch, 0, stream, dev)), flush=True)
