"""Point profiles/current.json (bench.py's cross-check index) at freshly committed profiles.

    python tools/profile_index.py HASH [rocprof_stats=PATH] [coatt_trace=PATH] [pmc=PATH]

HASH = the source hash of the library the profiles were taken with (the `build.lib_source_hash`
field of that pass's bench JSON line).  Entries not named keep their previous path; bench.py marks
any field read from an entry stale when the library it loads has another hash.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IDX = os.path.join(REPO, "profiles", "current.json")


def main(argv):
    if not argv:
        raise SystemExit(__doc__)
    try:
        with open(IDX) as f:
            idx = json.load(f)
    except (OSError, ValueError):
        idx = {}
    idx["lib_source_hash"] = argv[0]
    for a in argv[1:]:
        k, v = a.split("=", 1)
        if k not in ("rocprof_stats", "coatt_trace", "pmc"):
            raise SystemExit("unknown entry " + k)
        if not os.path.exists(os.path.join(REPO, v)):
            raise SystemExit("no such file " + v)
        idx[k] = v
    with open(IDX, "w") as f:
        json.dump(idx, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:])
