"""MI355X-native visual-onomatopoeia -> mel -> 22.05 kHz waveform synthesis path.

The host side mirrors the reference's Python surface (``model``, ``transformer``,
``hifigan``, ``utils.model``, ``utils.tools``); every tensor op on the path runs
in hand-written HIP kernels for gfx950 behind the C ABI in ``include/vonoma.h``
(``csrc/`` -> ``lib/libvonoma.so``).  See DESIGN.md.
"""

import os as _os
import sys as _sys

# HIP-graph training replays need the CLR's ordinary graph-launch path: with "packet capture"
# (the ROCm default) replays of the training step computed wrong values on this runtime
# (train.py).  Read once when the HIP runtime initialises: effective when
# this package is imported before the first CUDA call (an explicit user setting wins).  When the
# package sets it itself after torch has already initialised the runtime, the setting is dead:
# recorded here, and train._check_graph_runtime refuses graphed training in that case.
_PC = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"
PACKET_CAPTURE_SET_LATE = False
if _PC not in _os.environ:
    _torch = _sys.modules.get("torch")
    try:
        PACKET_CAPTURE_SET_LATE = bool(_torch is not None and _torch.cuda.is_initialized())
    except Exception:  # a partially imported torch
        PACKET_CAPTURE_SET_LATE = False
    _os.environ[_PC] = "0"

__version__ = "0.2.0"
