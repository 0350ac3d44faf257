from .Models import Encoder, Decoder, get_sinusoid_encoding_table  # noqa: F401
from .Layers import PostNet, FFTBlock  # noqa: F401
