"""Run an unmodified reference attack script on the MI355X path.

    cd /path/to/Audio-Backdoor-Attack
    PYTHONPATH=/path/to/repo python -m abd_amd.run badnets.py --model smallcnn ...
    PYTHONPATH=/path/to/repo python -m abd_amd.run --config config/badnets.yaml badnets.py [...]

``python script.py`` puts the script's directory at sys.path[0], where the reference's own
``prepare_dataset.py`` and ``utils/`` would win over anything on PYTHONPATH.  This runner builds
the path the drop-in needs -- ``dropin/`` first, then the script directory, then the rest -- and
executes the script as ``__main__`` with its own argv.  Modules the drop-in provides
(prepare_dataset, utils.training_tools, utils.models, the trigger modules) resolve to abd_amd;
the rest of ``utils`` (visual_tools) falls through to the reference (dropin/utils/__init__.py).

``--config file.yaml``: the reference ships per-attack YAML files (config/*.yaml) but no
script reads them (``# import yaml`` is commented out, fp.py:12).  The runner reads one with
``yaml.safe_load`` and makes its keys the DEFAULTS of the script's own argparse parser when the
script parses its arguments -- flags given on the command line still win, keys the parser does not
define are reported on stderr and ignored, ``num_epoches`` (the YAML spelling) maps to
``--num_epochs``.  Values keep their YAML types, so ``load_clean_data: False`` is False (the
script's ``type=bool`` flag would turn the STRING "False" into True).
"""
from __future__ import annotations

import argparse
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


YAML_ALIASES = {"num_epoches": "num_epochs"}   # config/*.yaml spelling -> the scripts' flag


def load_config(path: str) -> dict:
    """config/*.yaml -> {argparse dest: value} (safe loader: the file is data, never code)."""
    import yaml
    with open(path) as f:
        data = yaml.safe_load(f) or {}
    if not isinstance(data, dict):
        raise SystemExit(f"{path}: expected a mapping of argument names to values")
    return {YAML_ALIASES.get(k, k): v for k, v in data.items()}


class config_defaults:
    """While active, every ArgumentParser.parse_args / parse_known_args first takes `values` as the
    defaults of the destinations the parser defines (command-line flags still override them)."""

    def __init__(self, values: dict, source: str = "config"):
        self.values, self.source = dict(values), source

    def __enter__(self):
        self._orig = argparse.ArgumentParser.parse_known_args
        values, source, orig = self.values, self.source, self._orig

        def parse_known_args(parser, args=None, namespace=None):
            dests = {a.dest for a in parser._actions}
            known = {k: v for k, v in values.items() if k in dests}
            unknown = sorted(k for k in values if k not in dests)
            if unknown and not getattr(parser, "_abd_config_noted", False):
                print(f"abd_amd.run: {source}: no such argument in this script, ignored: {', '.join(unknown)}",
                      file=sys.stderr)
                parser._abd_config_noted = True
            parser.set_defaults(**known)
            return orig(parser, args, namespace)
        argparse.ArgumentParser.parse_known_args = parse_known_args   # parse_args goes through it
        return self

    def __exit__(self, *exc):
        argparse.ArgumentParser.parse_known_args = self._orig
        return False


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    cfg = None
    if argv[:1] == ["--config"]:
        if len(argv) < 2:
            raise SystemExit("--config needs a YAML file")
        cfg, argv = argv[1], argv[2:]
    if not argv:
        raise SystemExit("usage: python -m abd_amd.run [--config config/<attack>.yaml] <attack_script.py> [script args...]")
    script = argv[0]
    setup_path(script)
    sys.argv = [script] + argv[1:]
    if cfg is None:
        runpy.run_path(script, run_name="__main__")
        return
    with config_defaults(load_config(cfg), cfg):
        runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
