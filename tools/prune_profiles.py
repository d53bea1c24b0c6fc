#!/usr/bin/env python3
"""Keep in profiles/ only what is read or cited; archive the rest.

Kept:
  * every pmc_*.json record that bench.py's selectors (latest_pmc / latest_conv_pmc /
    latest_inplace_pmc) return for some query the benchmark can make with this library (build
    variants from tests/conftest.py's BUILD_VARIANTS, tile orders 0/1, zero window 0/1, the
    row-band records, both pyramid backings);
  * every profiles/<file> that DESIGN.md, README.md or INTEGRATION.md names;
  * files matching --keep patterns (e.g. this round's _r05 logs).
Everything else is moved into profiles/archive_r01-r04.tar.xz (tracked; listed in .gpurunignore,
so it never travels to a GPU box), appended to if it exists.
    python3 tools/prune_profiles.py [--dry-run] [--keep GLOB ...]
"""
import argparse
import fnmatch
import json
import os
import re
import subprocess
import sys
import tarfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
PDIR = os.path.join(REPO, "profiles")
ARCHIVE = "archive_r01-r04.tar.xz"


def selected_pmc():
    import functools
    import io

    import bench
    from conftest import BUILD_VARIANTS

    # the selectors re-read every record per query: serve them from memory
    @functools.lru_cache(maxsize=None)
    def _text(path):
        with open(path) as fh:
            return fh.read()
    bench.open = lambda path, *a, **k: io.StringIO(_text(path))
    listing = sorted(os.listdir(PDIR))
    bench.os = type("os_cached", (), {"path": os.path, "listdir": staticmethod(lambda d: list(listing)),
                                      "environ": os.environ})

    keep = set()
    recs = {}
    for f in sorted(os.listdir(PDIR)):
        if f.startswith("pmc_") and f.endswith(".json"):
            try:
                with open(os.path.join(PDIR, f)) as fh:
                    recs[f] = json.load(fh)
            except (OSError, ValueError):
                continue
    seen = set()
    for rec in recs.values():
        cfg, op = rec.get("config"), rec.get("op", "build")
        if op in ("build", "subset"):
            if (cfg, op, rec.get("band_of")) in seen:
                continue
            seen.add((cfg, op, rec.get("band_of")))
            for v in BUILD_VARIANTS:
                for t in (0, 1):
                    for zw in (0, 1):
                        for ck in (2048, 0, None):
                            r = bench.latest_pmc(cfg, v, t, op=op, zero_window=zw, band_of=rec.get("band_of"),
                                                 chunk_kb=ck)
                            if r:
                                keep.add(r["file"])
        elif op == "conv":
            r = bench.latest_conv_pmc(cfg, {k: rec.get(k) for k in ("conv_kernel", "conv_rows", "conv_order")})
            if r:
                keep.add(r["file"])
        elif op in ("regen", "gauss"):
            key = "inplace_sub" if op == "regen" else "window_sub"
            r = bench.latest_inplace_pmc(cfg, op, {key: rec.get(key), "zero_window": rec.get("zero_window", 0)})
            if r:
                keep.add(r["file"])
    return keep


def cited():
    names = set(os.listdir(PDIR))
    keep = set()
    for doc in ("DESIGN.md", "README.md", "INTEGRATION.md"):
        path = os.path.join(REPO, doc)
        if not os.path.exists(path):
            continue
        text = open(path).read()
        for m in re.finditer(r"profiles/([A-Za-z0-9_.{},*\-]+)", text):
            ref = m.group(1).rstrip(".,)")
            # brace sets like bench_{default,c3}_r04aj.log and globs like timed_dispatches_c2_*
            alts = [ref]
            b = re.search(r"\{([^}]*)\}", ref)
            if b:
                alts = [ref[:b.start()] + x + ref[b.end():] for x in b.group(1).split(",")]
            for a in alts:
                keep.update(n for n in names if fnmatch.fnmatch(n, a) or n == a)
        # bare file names in backticks (the tables cite `bench_c3_r04aa.log` without the directory)
        for m in re.finditer(r"`([A-Za-z0-9_.{},*\-]+\.(?:log|json|csv|txt))`", text):
            ref = m.group(1)
            alts = [ref]
            b = re.search(r"\{([^}]*)\}", ref)
            if b:
                alts = [ref[:b.start()] + x + ref[b.end():] for x in b.group(1).split(",")]
            for a in alts:
                keep.update(n for n in names if fnmatch.fnmatch(n, a))
    return keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--keep", nargs="*", default=[])
    args = ap.parse_args()
    names = sorted(n for n in os.listdir(PDIR) if os.path.isfile(os.path.join(PDIR, n)))
    keep = selected_pmc() | cited() | {ARCHIVE, "pmc_records.json"}
    for pat in args.keep:
        keep.update(n for n in names if fnmatch.fnmatch(n, pat))
    drop = [n for n in names if n not in keep]
    # the kept PMC records go into ONE file bench.py reads (bench.pmc_records), not hundreds
    gather = sorted(n for n in keep & set(names) if n.startswith("pmc_") and n.endswith(".json") and n != "pmc_records.json")
    print(f"{len(names)} files: keep {len(names) - len(drop)} ({len(gather)} PMC records gathered into "
          f"pmc_records.json), archive {len(drop)}")
    if args.dry_run:
        for n in sorted(keep & set(names)):
            print("  keep", n)
        return
    if gather:
        agg = os.path.join(PDIR, "pmc_records.json")
        recs = json.load(open(agg)) if os.path.exists(agg) else []
        have = {r["file"] for r in recs}
        for n in gather:
            rec = json.load(open(os.path.join(PDIR, n)))
            if n not in have:
                recs.append(dict(rec, file=n))
        recs.sort(key=lambda r: r["file"])
        with open(agg, "w") as fh:
            json.dump(recs, fh, indent=0, sort_keys=True)
            fh.write("\n")
        subprocess.run(["git", "rm", "-q", "--cached", "--ignore-unmatch", *[os.path.join("profiles", n) for n in gather]],
                       cwd=REPO, check=True)
        for n in gather:
            os.remove(os.path.join(PDIR, n))
    if not drop:
        return
    apath = os.path.join(PDIR, ARCHIVE)
    members = {}
    if os.path.exists(apath):
        with tarfile.open(apath, "r:xz") as t:
            for m in t.getmembers():
                members[m.name] = t.extractfile(m).read() if m.isfile() else None
    for n in drop:
        with open(os.path.join(PDIR, n), "rb") as fh:
            members[n] = fh.read()
    tmp = apath + ".tmp"
    import io
    with tarfile.open(tmp, "w:xz") as t:
        for name in sorted(members):
            data = members[name]
            if data is None:
                continue
            info = tarfile.TarInfo(name)
            info.size = len(data)
            t.addfile(info, io.BytesIO(data))
    os.replace(tmp, apath)
    subprocess.run(["git", "rm", "-q", "--cached", "--ignore-unmatch", *[os.path.join("profiles", n) for n in drop]],
                   cwd=REPO, check=True)
    for n in drop:
        os.remove(os.path.join(PDIR, n))
    print(f"archived into profiles/{ARCHIVE} ({os.path.getsize(apath) / 1e6:.1f} MB)")


if __name__ == "__main__":
    main()
