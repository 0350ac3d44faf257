"""MI355X-native visual-onomatopoeia -> mel -> 22.05 kHz waveform synthesis path.

The host side mirrors the reference's Python surface (``model``, ``transformer``,
``hifigan``, ``utils.model``, ``utils.tools``); every tensor op on the path runs
in hand-written HIP kernels for gfx950 behind the C ABI in ``include/vonoma.h``
(``csrc/`` -> ``lib/libvonoma.so``).  See DESIGN.md.
"""

import os as _os

# HIP-graph training replays need the CLR's ordinary graph-launch path: with "packet capture"
# (the ROCm default) replays of the training step computed wrong values on this runtime
# (train.py).  Read once when the HIP runtime initialises: effective when
# this package is imported before the first CUDA call (an explicit user setting wins).
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

__version__ = "0.2.0"
