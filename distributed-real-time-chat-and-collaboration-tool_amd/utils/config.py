"""Config files for the CLIs (SURVEY §5 "Config / flags").

The reference hardcodes everything but ``--node-id/--port`` (server) and
``--server`` (client).  Here every entry point's flags can also come from a
JSON or YAML file (``--config node1.yaml``); values on the command line
override the file, and the file overrides the built-in defaults (which equal
the reference's values where the reference has one).  Keys are
the flags' destination names, e.g. ``node_id``, ``election_timeout``,
``snapshot_every``; an unknown key is an error, not silently ignored.
YAML is read with ``yaml.safe_load`` (no object construction).
"""
from __future__ import annotations

import argparse
import json
import os


def load_file(path: str) -> dict:
    with open(path) as f:
        text = f.read()
    if os.path.splitext(path)[1].lower() in (".yaml", ".yml"):
        import yaml

        data = yaml.safe_load(text) or {}
    else:
        data = json.loads(text or "{}")
    if not isinstance(data, dict):
        raise ValueError(f"{path}: top level must be a mapping")
    return data


def parse_with_config(ap: argparse.ArgumentParser, argv=None) -> argparse.Namespace:
    """``ap.parse_args`` with a ``--config FILE`` layer between the defaults
    and the command line."""
    ap.add_argument("--config", default=None, metavar="FILE",
                    help="JSON/YAML file of flag values (command-line flags override it)")
    pre_ap = argparse.ArgumentParser(add_help=False)
    pre_ap.add_argument("--config", default=None)
    pre, _ = pre_ap.parse_known_args(argv)
    if pre.config:
        values = load_file(pre.config)
        dests = {a.dest for a in ap._actions}
        unknown = sorted(k for k in values if k.replace("-", "_") not in dests)
        if unknown:
            ap.error(f"{pre.config}: unknown keys {unknown}")
        ap.set_defaults(**{k.replace("-", "_"): v for k, v in values.items()})
        # a required flag satisfied by the file is no longer required
        for a in ap._actions:
            if a.required and a.dest in {k.replace("-", "_") for k in values}:
                a.required = False
    return ap.parse_args(argv)
