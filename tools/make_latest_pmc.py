"""Merge a tools/pmc_summary.py entry into profiles/latest_pmc.json (read by bench.py).

usage: python tools/make_latest_pmc.py <entry.json> <source label>
An entry for the same config replaces the old one (bench.py attaches an entry
only to a library whose zrt_build_id() equals the entry's build_id).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, label = sys.argv[1], sys.argv[2]
    with open(src) as f:
        e = json.load(f)
    e["source"] = label
    assert e.get("build_id"), "entry without build_id (bench line older than round 3?)"
    path = os.path.join(REPO, "profiles", "latest_pmc.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    entries = [x for x in d.get("entries", []) if x.get("config") != e["config"]]
    entries.append(e)
    with open(path, "w") as f:
        json.dump({"entries": entries}, f, indent=1)
    print(f"{len(entries)} entries in {path}")


if __name__ == "__main__":
    main()
