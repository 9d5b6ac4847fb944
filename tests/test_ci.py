"""The short CI run (travis.sh, the counterpart of the reference's
travis.sh:9-24 + Jenkinsfile:28-91): run_simulations on the local job manager
-> monitor_func_test regex oracle -> get_stats -> plot-correlation against the
committed statistics archive -> exact per-kernel regression gate."""
import csv
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "ci", "golden_QV100-SASS_rodinia_2.0-ft.csv")


def _ci(tmp_path, golden, apps="nn,pathfinder"):
    env = dict(os.environ, CI_SKIP_BUILD="1", CI_APPS=apps, CI_WORK=str(tmp_path / "ci_run"), CI_GOLDEN=golden,
               CI_NAME="pytest-ci")
    return subprocess.run(["bash", os.path.join(ROOT, "travis.sh")], env=env, capture_output=True, text=True,
                          timeout=600, cwd=ROOT)


def test_travis_short_run_matches_archive(native, tmp_path):
    r = _ci(tmp_path, GOLDEN)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "All jobs passed" in r.stdout
    assert "cycle MAE vs archive 0.000 %, 0 failures" in r.stdout
    assert "Cycles" in r.stdout and "MAE=   0.00%" in r.stdout  # the correlator ran on the archive


def test_travis_gate_catches_drift(native, tmp_path):
    rows = list(csv.DictReader(open(GOLDEN)))
    for r in rows:
        if r["app"].startswith("nn-"):
            r["cycles"] = str(int(r["cycles"]) + 100)
    bad = tmp_path / "drifted.csv"
    with open(bad, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    r = _ci(tmp_path, str(bad))
    assert r.returncode != 0
    assert "FAIL nn-rodinia-2.0-ft" in r.stdout
