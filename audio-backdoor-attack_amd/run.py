"""Run an unmodified reference attack script on the MI355X path.

    cd /path/to/Audio-Backdoor-Attack
    PYTHONPATH=/path/to/repo python -m abd_amd.run badnets.py --model smallcnn ...

``python script.py`` puts the script's directory at sys.path[0], where the reference's own
``prepare_dataset.py`` and ``utils/`` would win over anything on PYTHONPATH.  This runner builds
the path the drop-in needs -- ``dropin/`` first, then the script directory, then the rest -- and
executes the script as ``__main__`` with its own argv.  Modules the drop-in provides
(prepare_dataset, utils.training_tools, utils.models, the trigger modules) resolve to abd_amd;
the rest of ``utils`` (visual_tools) falls through to the reference (dropin/utils/__init__.py).
"""
from __future__ import annotations

import os
import runpy
import sys

DROPIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dropin")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def setup_path(script: str) -> None:
    script_dir = os.path.dirname(os.path.abspath(script))
    rest = [p for p in sys.path if os.path.abspath(p or os.getcwd()) not in (DROPIN, script_dir)]
    sys.path[:] = [DROPIN, script_dir] + rest + ([ROOT] if ROOT not in rest else [])
    os.environ["ABD_REFERENCE_ROOT"] = script_dir   # the only utils/ the drop-in falls through to
    for name in [m for m in sys.modules if m in ("utils", "prepare_dataset") or m.startswith("utils.")]:
        del sys.modules[name]   # a stale reference import must not shadow the drop-in


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        raise SystemExit("usage: python -m abd_amd.run <attack_script.py> [script args...]")
    script = argv[0]
    setup_path(script)
    sys.argv = [script] + argv[1:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
