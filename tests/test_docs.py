"""The evidence trail resolves: every profiles/ file DESIGN.md, README.md and
INTEGRATION.md cite — by path or as a backticked file name, brace sets and globs expanded — is a
tracked file under profiles/, and the directory stays small."""
import fnmatch
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _expand(ref):
    b = re.search(r"\{([^}]*)\}", ref)
    if not b:
        return [ref]
    out = []
    for x in b.group(1).split(","):
        out += _expand(ref[:b.start()] + x + ref[b.end():])
    return out


def _cited(text):
    refs = set()
    for m in re.finditer(r"profiles/([A-Za-z0-9_.{},*<>\-]+)", text):
        refs.add(re.sub(r"<[^>]*>", "*", m.group(1).rstrip(".,)")))  # <V> placeholders: any text
    for m in re.finditer(r"`([A-Za-z0-9_{},*\-]+(?:\.[a-z0-9]+)*\.(?:log|json|csv))`", text):
        refs.add(m.group(1))
    return refs


def _missing(doc, names):
    text = open(os.path.join(REPO, doc)).read()
    out = []
    for ref in _cited(text):
        if ref.startswith(("pmc_records.json#", "archive_")) or "/" in ref.rstrip("/"):
            continue
        if ref.endswith(".json") and not ref.startswith(("pmc_", "sq_", "calib_")):
            continue  # repo-level JSON (BENCH_r05.json, meta.json, ...) is not a profile
        for alt in _expand(ref):
            if not any(fnmatch.fnmatch(n, alt) for n in names):
                out.append((doc, alt))
    return out


def _profile_names():
    import json  # PMC records gathered into profiles/pmc_records.json keep their file names

    tracked = subprocess.run(["git", "ls-files", "profiles"], cwd=REPO, capture_output=True, text=True,
                             check=True).stdout.split()
    names = {os.path.relpath(p, "profiles") for p in tracked} | set(os.listdir(os.path.join(REPO, "profiles")))
    with open(os.path.join(REPO, "profiles", "pmc_records.json")) as f:
        names |= {r["file"] for r in json.load(f)}
    return names


def test_every_cited_profile_exists():
    names = _profile_names()
    missing = []
    for doc in ("DESIGN.md", "README.md", "INTEGRATION.md"):
        missing += _missing(doc, names)
    assert not missing, missing


def test_design_history_citations_resolve_to_profiles_or_the_archive():
    """DESIGN_HISTORY.md cites round 1-4 logs that the round-5 prune moved into
    profiles/archive_r01-r04.tar.xz; every citation is a current profile or an archive member."""
    import tarfile

    with tarfile.open(os.path.join(REPO, "profiles", "archive_r01-r04.tar.xz")) as t:
        archived = {os.path.basename(m.name) for m in t.getmembers()}
    missing = _missing("DESIGN_HISTORY.md", _profile_names() | archived)
    assert not missing, missing


def test_profiles_directory_stays_small():
    tracked = subprocess.run(["git", "ls-files", "profiles"], cwd=REPO, capture_output=True, text=True,
                             check=True).stdout.split()
    assert len(tracked) < 400, len(tracked)


def _bench_records():
    import glob
    import json

    out = {}
    for p in glob.glob(os.path.join(REPO, "BENCH_r*.json")):
        m = re.search(r"BENCH_r(\d+)\.json$", p)
        if m:
            with open(p) as f:
                out[int(m.group(1))] = (os.path.basename(p), json.load(f))
    return out


def _last_commit_time(path):
    r = subprocess.run(["git", "log", "-1", "--format=%ct", "--", path], cwd=REPO, capture_output=True, text=True)
    return int(r.stdout.strip() or 0)


def test_quoted_driver_headline_is_the_newest_record():
    """DESIGN.md and README.md quote the driver's headline from the newest
    BENCH_r*.json — its name, % of the roofline, kernel_ms, Mpix/s and CPU baseline as the driver
    recorded them.  (A record the driver commits after the docs' last change may be one round
    newer than the one they cite.)"""
    recs = _bench_records()
    if not recs:
        return
    newest = max(recs)
    for doc in ("DESIGN.md", "README.md"):
        text = open(os.path.join(REPO, doc)).read()
        m = re.search(r"driver[^\n]*?\(`(BENCH_r(\d+)\.json)`", text)
        assert m, (doc, "names no driver record")
        cited = int(m.group(2))
        if cited != newest:
            assert cited == newest - 1 and _last_commit_time(recs[newest][0]) >= _last_commit_time(doc), \
                (doc, "cites", m.group(1), "newest", recs[newest][0])
        name, rec = recs[cited]
        p = rec["parsed"]
        want = [f"{100 * p['roofline']['frac']:.1f} %", f"{p['roofline']['kernel_ms']:.4f}",
                f"{round(p['value']):,}", f"{p['cpu_baseline']['value']:,.1f}"]
        for w in want:
            assert w in text, (doc, name, w)
