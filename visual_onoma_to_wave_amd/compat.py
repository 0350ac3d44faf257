"""Drop-in import aliases for the reference's module names.

The reference is imported two ways: with the ``scripts.`` prefix
(``prediction.ipynb``: ``from scripts.utils.model import get_model, get_vocoder``) and,
after ``sys.path.append("./scripts")``, as top-level packages (``04_train.py``:
``from utils.model import get_model``, ``from model import FastSpeech2Loss``;
internally ``import transformer``, ``import hifigan``).  ``install()`` registers this
package's modules under all of those names, so the callers run unchanged:

    import visual_onoma_to_wave_amd.compat as c; c.install()
"""

import importlib
import sys

_PKG = __name__.rsplit(".", 1)[0]

_MAP = {
    "model": "model",
    "model.vtts": "model.vtts",
    "model.modules": "model.modules",
    "model.loss": "model.loss",
    "model.optimizer": "model.optimizer",
    "model.visual_feature_extractor": "model.visual_feature_extractor",
    "transformer": "transformer",
    "transformer.Models": "transformer.Models",
    "transformer.Layers": "transformer.Layers",
    "transformer.SubLayers": "transformer.SubLayers",
    "transformer.Modules": "transformer.Modules",
    "transformer.Constants": "transformer.Constants",
    "hifigan": "hifigan",
    "hifigan.models": "hifigan.models",
    "utils": "utils",
    "utils.model": "utils.model",
    "utils.tools": "utils.tools",
    "utils.symbols": "utils.symbols",
    "audio": "audio",
    "dataset": "dataset",
}


def install(prefixes=("", "scripts.")):
    """Alias ``<prefix><name>`` -> ``visual_onoma_to_wave_amd.<name>`` in sys.modules."""
    if "scripts." in prefixes and "scripts" not in sys.modules:
        import types
        pkg = types.ModuleType("scripts")
        pkg.__path__ = []
        sys.modules["scripts"] = pkg
    for alias, target in _MAP.items():
        try:
            mod = importlib.import_module(f"{_PKG}.{target}")
        except ImportError:
            continue
        for pre in prefixes:
            sys.modules[pre + alias] = mod
            parent, _, leaf = (pre + alias).rpartition(".")
            if parent and parent in sys.modules:
                setattr(sys.modules[parent], leaf, mod)
    return sys.modules[_PKG]
