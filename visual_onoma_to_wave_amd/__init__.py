"""MI355X-native visual-onomatopoeia -> mel -> 22.05 kHz waveform synthesis path.

The host side mirrors the reference's Python surface (``model``, ``transformer``,
``hifigan``, ``utils.model``, ``utils.tools``); every tensor op on the path runs
in hand-written HIP kernels for gfx950 behind the C ABI in ``include/vonoma.h``
(``csrc/`` -> ``lib/libvonoma.so``).  See DESIGN.md.
"""

__version__ = "0.1.0"
