"""Config 4 block by block (64 channels x 4096-sample blocks, 131072-tap Large
Church IR[c mod 2]) through ad_conv_multi_stream_process_block_device, for a
kernel trace: `rocprofv3 --kernel-trace --stats -- python3 tools/stream64_probe.py`."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from algodsp import conv, irlib, signals  # noqa: E402

C, B, nb = 64, 4096, int(sys.argv[1]) if len(sys.argv) > 1 else 64
ir = irlib.large_church()
s = conv.MultiChannelStreamingConvolver(ir, B, C, ir_index=[c % 2 for c in range(C)])
dx = torch.from_numpy(np.stack([signals.white_noise(B, 0x5EED + c) for c in range(C)])).cuda()
dy = torch.empty_like(dx)
st = torch.cuda.current_stream().cuda_stream
for _ in range(8):
    s.process_block_device(dx.data_ptr(), B, dy.data_ptr(), B, st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(nb):
    s.process_block_device(dx.data_ptr(), B, dy.data_ptr(), B, st)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / nb
print(f"{dt * 1e6:.1f} us per block, {C * B / dt / 1e9:.2f} Gsamples/s")
