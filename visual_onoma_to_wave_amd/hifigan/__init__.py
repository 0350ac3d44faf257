from .models import Generator  # noqa: F401


class AttrDict(dict):
    """dict with attribute access (reference: scripts/hifigan/__init__.py:4-7)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


def __getattr__(name):
    # training-side modules (config C5) load on first use
    if name in ("MultiPeriodDiscriminator", "MultiScaleDiscriminator", "DiscriminatorP", "DiscriminatorS",
                "feature_loss", "discriminator_loss", "generator_loss", "MelLoss",
                "MultiResolutionSTFTLoss"):
        from . import discriminators
        return getattr(discriminators, name)
    if name == "HifiGanTrainer":
        from .train import HifiGanTrainer
        return HifiGanTrainer
    raise AttributeError(name)
