"""Drop-in import aliases for the reference's module names.

The reference is imported two ways: with the ``scripts.`` prefix
(``prediction.ipynb``: ``from scripts.utils.model import get_model, get_vocoder``) and,
after ``sys.path.append("./scripts")``, as top-level packages (``04_train.py``:
``from utils.model import get_model``, ``from model import FastSpeech2Loss``;
internally ``import transformer``, ``import hifigan``).  ``install()`` registers this
package's modules under all of those names, so the callers run unchanged:

    import visual_onoma_to_wave_amd.compat as c; c.install()

The hot-path names of ``utils.tools`` / ``utils.model`` (``to_device``,
``get_mask_from_lengths``, ``pad``, ``expand``, ``get_model``, ``vocoder_infer`` ...) are this
package's.  The callers also import helpers that are not on the path and are not built here --
``log`` / ``synth_one_sample`` (``scripts/04_train.py:12``, ``scripts/evaluate.py:10``) and
``plot_mel`` (``prediction.ipynb:215``), TensorBoard logging and matplotlib plotting.  Those
resolve to the CALLER'S OWN definitions: a name the build's module lacks is looked up in the
caller's ``scripts/utils/<module>.py``, executed once as a private module
(``utils._caller_tools``) whose relative imports (``from .model import vocoder_infer``,
``tools.py:224``) land on this package again.  The caller's tree is found from
``install(caller_root=...)``, ``$VO_CALLER_ROOT``, the working directory (the reference runs
from its repo root: ``scripts/hifigan/config.json`` is cwd-relative, ``utils/model.py:57``) or a
``.../scripts`` entry of ``sys.path`` (``04_train.py`` runs with its own directory first).
"""

import importlib
import importlib.util
import os
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

_caller_root = None          # set by install(caller_root=...)
_caller_mods = {}            # "utils.tools" -> the caller's module (executed once)
_caller_errors = {}          # "utils.tools" -> the exception its execution raised (not retried)


def install(prefixes=("", "scripts."), caller_root=None):
    """Alias ``<prefix><name>`` -> ``visual_onoma_to_wave_amd.<name>`` in sys.modules.

    ``caller_root``: the reference checkout whose ``scripts/`` tree supplies the non-path
    helpers (default: ``$VO_CALLER_ROOT``, the cwd, or a ``scripts`` dir on ``sys.path``)."""
    global _caller_root
    if caller_root is not None:
        _caller_root = os.fspath(caller_root)
    _caller_mods.clear()
    _caller_errors.clear()
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


def _scripts_dirs():
    """Candidate ``scripts/`` directories of the caller's checkout, in priority order."""
    roots = [r for r in (_caller_root, os.environ.get("VO_CALLER_ROOT"), os.getcwd()) if r]
    out = [os.path.join(r, "scripts") for r in roots]
    out += [p for p in sys.path if p and os.path.basename(os.path.normpath(p)) == "scripts"]
    pkg_dir = os.path.dirname(os.path.abspath(__file__))
    seen, res = set(), []
    for d in out:
        d = os.path.abspath(d)
        if d not in seen and not d.startswith(pkg_dir):
            seen.add(d)
            res.append(d)
    return res


def _load_caller(modname):
    """Execute the caller's own ``scripts/<modname>.py`` once as ``<pkg>._caller_<leaf>``."""
    if modname in _caller_mods:
        return _caller_mods[modname]
    rel = modname.replace(".", os.sep) + ".py"
    path = next((os.path.join(d, rel) for d in _scripts_dirs()
                 if os.path.isfile(os.path.join(d, rel))), None)
    if modname in _caller_errors:  # a failed execution is not retried on every attribute probe
        raise _caller_errors[modname]
    mod = None
    if path is not None:
        pkg, _, leaf = modname.rpartition(".")
        # relative imports of the caller's file ("from .model import vocoder_infer") resolve
        # against the aliased package, i.e. back onto this build
        if pkg and pkg not in sys.modules and f"scripts.{pkg}" in sys.modules:
            pkg = f"scripts.{pkg}"
        name = f"{pkg}._caller_{leaf}" if pkg else f"_caller_{leaf}"
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        try:
            spec.loader.exec_module(mod)
        except BaseException as e:  # SystemExit / KeyboardInterrupt too: no half-initialised module stays
            del sys.modules[name]
            if isinstance(e, Exception):  # only ordinary errors are remembered (not retried)
                _caller_errors[modname] = e
            raise
    _caller_mods[modname] = mod
    return mod


# names off the synthesis path that the caller's own utils files provide (reference
# scripts/utils/tools.py, scripts/utils/model.py); any other missing name is an AttributeError
# without executing the caller's file
CALLER_NAMES = {
    "utils.tools": {"to_device_synth", "log", "synth_one_sample", "plot_mel_withinput", "synth_samples",
                    "synth_for_eval", "synth_for_eval_strech", "synth_for_eval_continue", "plot_mel",
                    "pad_2D_image", "save_figure_to_numpy", "plot_alignment_to_numpy"},
    "utils.model": set(),
}


def caller_attr(modname, name):
    """``name`` from the caller's own ``scripts/<modname>.py`` (module ``__getattr__`` hook of
    ``utils.tools`` / ``utils.model``) for the names in ``CALLER_NAMES``.  Always AttributeError
    otherwise -- also when executing the caller's file failed (an optional import it needs is
    missing), so ``hasattr`` / ``getattr(..., default)`` probes stay probes; the failure is
    remembered and chained, not re-executed."""
    allowed = CALLER_NAMES.get(modname)
    if name.startswith("__") or (allowed is not None and name not in allowed):
        raise AttributeError(f"module '{modname}' has no attribute '{name}'")
    try:
        mod = _load_caller(modname)
    except Exception as e:
        raise AttributeError(f"module '{modname}' has no attribute '{name}': executing the caller's "
                             f"scripts/{modname.replace('.', '/')}.py failed ({type(e).__name__}: {e})") from e
    if mod is None or not hasattr(mod, name):
        raise AttributeError(
            f"module '{modname}' has no attribute '{name}': it is not on the synthesis path "
            f"(not built by {_PKG}) and no caller tree provides it (looked in "
            f"{[os.path.join(d, modname.replace('.', os.sep) + '.py') for d in _scripts_dirs()]}; "
            f"pass compat.install(caller_root=...) or set VO_CALLER_ROOT)")
    return getattr(mod, name)
