"""tinycudann -- MI355X (gfx950) drop-in for the reference PyTorch bindings
(reference bindings/torch/tinycudann/__init__.py, modules.py).

The compute path is the HIP library lib/libtcnn_mi355x.so driven through its C-ABI
(include/tcnn_mi355x.h); PyTorch only provides device memory and the stream.
"""
from tinycudann._lib import TcnnError  # noqa: F401
from tinycudann.trainer import Trainer, create_from_config  # noqa: F401

try:
    from tinycudann.modules import Encoding, Network, NetworkWithInputEncoding, free_temporary_memory  # noqa: F401
except EnvironmentError as _e:  # no GPU: the reference raises at import time (modules.py:18-19)
    _err = _e

    def _unavailable(*args, **kwargs):
        raise _err

    Encoding = Network = NetworkWithInputEncoding = free_temporary_memory = _unavailable
