from .vtts import vTTS  # noqa: F401
from .loss import FastSpeech2Loss  # noqa: F401
from .optimizer import ScheduledOptim  # noqa: F401
