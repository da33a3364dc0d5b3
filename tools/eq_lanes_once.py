"""One K_lanes call at 256 channels x 2^20 samples (config 5's five EQ
sections), after a warm-up call: the launch rocprofv3 counter passes look at
(tools/eq_lanes_pmc.sh)."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
import torch

from algodsp import design, processors, signals

fs = 48000.0
C_, n = 256, 1 << 20
fx = processors.EffectChain(C_, design.config5_eq(fs), None, None, fs)
x = torch.from_numpy(0.5 * signals.white_noise(C_ * n, 3).reshape(C_, n)).cuda()
s = torch.cuda.current_stream().cuda_stream
for _ in range(2):
    fx.process_device(x.data_ptr(), n, n, s)
torch.cuda.synchronize()
print("engine", fx.LastEngine())
