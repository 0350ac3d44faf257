from .models import Generator  # noqa: F401


class AttrDict(dict):
    """dict with attribute access (reference: scripts/hifigan/__init__.py:4-7)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self
