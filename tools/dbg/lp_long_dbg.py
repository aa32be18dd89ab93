"""GPU debug: bf16 vs fp32 logits per sample at T_syb <= 128 and > 128 (which rows differ)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_lowp_state_gpu as TL  # noqa: E402
from savqa_amd.data import model_args, synthetic_batch  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402
from savqa_amd.utils import init_params_  # noqa: E402


def _model(prec, seed, Hm):
    return TL._model(prec, seed)


for Hm in (128,):
  for Ns in (59, 140):
    for B in (4, 8):
        b = synthetic_batch(B, Nv=36, Lq=14, Ns=Ns, topN=5, num_classes=60, seed=7, device="cuda")
        out = {}
        for mode in ("fp32", "bf16"):
            m = _model(mode, 3, Hm)
            m.eval()
            with torch.no_grad():
                r = m(*model_args(b), decMask=True, mcb=False)
            out[mode] = [x.clone() for x in r[:3]]
        for k, nm in enumerate(("concat", "vis", "syb")):
            a, c = out["bf16"][k].double(), out["fp32"][k].double()
            rowerr = ((a - c).norm(dim=1) / c.norm(dim=1)).tolist()
            # best-matching fp32 row for each bf16 row
            dist = torch.cdist(a, c)
            match = dist.argmin(1).tolist()
            print(f"Hm={Hm} Ns={Ns} B={B} {nm}: row err {[round(x, 3) for x in rowerr]} nearest fp32 row {match}")
