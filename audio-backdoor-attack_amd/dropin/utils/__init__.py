"""Drop-in ``utils`` package: the accelerated modules live here, everything else falls through.

The reference's ``utils/`` is a namespace directory next to the attack scripts.  This regular
package takes its place (``abd_amd.run`` puts ``dropin/`` first on ``sys.path``) and then extends
its ``__path__`` with every other ``utils`` directory on ``sys.path`` -- the reference checkout's
-- so modules that are not accelerated (``utils.visual_tools``'s plots, badnets.py:14) import
from the reference unchanged.
"""
import importlib.util
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))


def _other_portions():
    """The reference checkout's ``utils`` directory.  ``abd_amd.run`` names it (the attack
    script's directory, ABD_REFERENCE_ROOT); otherwise only a ``utils`` directory whose parent
    looks like the reference checkout (it holds ``prepare_dataset.py``) is taken, so an unrelated
    ``utils`` package on sys.path (site-packages, the CWD) is never executed in its place."""
    root = os.environ.get("ABD_REFERENCE_ROOT")
    if root:
        d = os.path.join(os.path.abspath(root), "utils")
        return [d] if os.path.isdir(d) and os.path.realpath(d) != os.path.realpath(_HERE) else []
    out = []
    for entry in sys.path:
        base = os.path.abspath(entry or os.getcwd())
        d = os.path.join(base, "utils")
        if (os.path.isdir(d) and os.path.isfile(os.path.join(base, "prepare_dataset.py"))
                and os.path.realpath(d) != os.path.realpath(_HERE) and d not in out):
            out.append(d)
    return out


for _d in _other_portions():
    if _d not in __path__:
        __path__.append(_d)


def reference_module(name: str):
    """The reference's own ``utils/<name>.py`` (a fall-through portion), loaded under a private
    name, or None when no reference checkout is on sys.path."""
    key = f"{__name__}._reference_{name}"
    if key in sys.modules:
        return sys.modules[key]
    for d in __path__[1:]:
        f = os.path.join(d, name + ".py")
        if os.path.isfile(f):
            spec = importlib.util.spec_from_file_location(key, f)
            mod = importlib.util.module_from_spec(spec)
            sys.modules[key] = mod
            spec.loader.exec_module(mod)
            return mod
    return None
