"""savqa_amd -- MI355X-native (gfx950) implementation of the SA-VQA model_v=3
structured-alignment hot path (Peixixiong/Structured-Alignment-VQA,
models/modules.py + models/AttModel_x3.py + the DDP step of
models/main_itp_ddp_tar_super_node.py).

Host code mirrors the reference's nn.Module API; the compute runs in libsavqa.so
(HIP kernels for CDNA4, C ABI in include/savqa.h) bound with ctypes.
"""
__version__ = "0.1.0"

from . import _lib  # noqa: F401


def __getattr__(name):  # lazy: importing the package must not need a GPU
    if name in ("AttModel",):
        from .AttModel_x3 import AttModel
        return AttModel
    if name == "Adam":
        from .optim import Adam
        return Adam
    if name == "smoothed_loss":
        from .loss import smoothed_loss
        return smoothed_loss
    raise AttributeError(name)
