"""End-to-end drop-in test: the reference's own bam-somaticsniper CLI (dual-BAM
pileup, FASTA, writers -- oracle/_ref, compiled from /root/reference) against
the same CLI re-linked with the batching shim over the C ABI
(integration/_build/bam-somaticsniper-amd).  Outputs must be
byte-identical for every output format and option set, on the reference's own
integration-test data (expected.vcf) and on synthetic BAM pairs (tests/bamgen.py).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_CLI = os.path.join(ROOT, "oracle", "_ref", "bam-somaticsniper")
AMD_CLI = os.path.join(ROOT, "integration", "_build", "bam-somaticsniper-amd")
ITEST = os.path.join(ROOT, "tests", "golden", "integration")

OPTSETS = [[], ["-Q", "0"], ["-J"], ["-J", "-s", "1e-5", "-Q", "5"], ["-p", "-Q", "0"],
           ["-L", "-G", "-Q", "0"], ["-T", "0.9", "-N", "3", "-r", "0.01"], ["-q", "20", "-Q", "0"]]
FORMATS = ["classic", "vcf", "bed"]

need_ref = pytest.mark.skipif(not os.path.exists(REF_CLI), reason="reference CLI not built (make -f oracle/ref.mk)")
need_amd = pytest.mark.skipif(not os.path.exists(AMD_CLI), reason="shim CLI not built (make -f integration/shim.mk)")


def strip_volatile(text):
    return "".join(l for l in text.splitlines(True) if not l.startswith("##fileDate"))


def run(cli, args, cwd, env=None):
    out = os.path.join(cwd, "out.txt")
    p = subprocess.run([cli] + args + [out], cwd=cwd, capture_output=True, text=True, timeout=600,
                       env=env)
    body = open(out).read() if os.path.exists(out) else None
    return p.returncode, body, p.stderr


@pytest.fixture(scope="module")
def bam_pairs(tmp_path_factory):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bamgen
    pairs = []
    for seed, kw in [(1, {}), (2, dict(depth_t=60, depth_n=30)), (3, dict(exotic=False, lengths=(5000,)))]:
        d = tmp_path_factory.mktemp(f"pair{seed}")
        bamgen.make_pair(str(d), seed=seed, **kw)
        pairs.append(str(d))
    return pairs


@need_ref
def test_reference_cli_on_integration_data(tmp_path):
    for f in os.listdir(ITEST):
        shutil.copy(os.path.join(ITEST, f), tmp_path)
    rc, body, _ = run(REF_CLI, ["-F", "vcf", "-f", "small.fa", "t-small.bam", "n-small.bam"], str(tmp_path))
    assert rc == 0
    expected = open(os.path.join(ITEST, "expected.vcf")).read()
    drop = ("##fileDate", "##reference")
    keep = lambda t: [l for l in t.splitlines() if not l.startswith(drop)]
    assert keep(body) == keep(expected)


@need_ref
def test_reference_cli_on_synthetic_bams(bam_pairs):
    for d in bam_pairs:
        rc, body, err = run(REF_CLI, ["-Q", "0", "-f", "ref.fa", "tumor.bam", "normal.bam"], d)
        assert rc == 0, err
        assert body.count("\n") > 5


@need_amd
def test_shim_cli_fails_loudly_without_gpu(tmp_path):
    """No CPU fallback: without a usable GPU the shim exits non-zero with a message."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    for f in os.listdir(ITEST):
        shutil.copy(os.path.join(ITEST, f), tmp_path)
    rc, _, err = run(AMD_CLI, ["-f", "small.fa", "t-small.bam", "n-small.bam"], str(tmp_path))
    assert rc != 0 and "sniper_amd shim" in err


@pytest.mark.gpu
@need_ref
@need_amd
def test_shim_integration_expected_vcf(tmp_path):
    for f in os.listdir(ITEST):
        shutil.copy(os.path.join(ITEST, f), tmp_path)
    rc, body, err = run(AMD_CLI, ["-F", "vcf", "-f", "small.fa", "t-small.bam", "n-small.bam"], str(tmp_path))
    assert rc == 0, err
    expected = open(os.path.join(ITEST, "expected.vcf")).read()
    drop = ("##fileDate", "##reference")
    keep = lambda t: [l for l in t.splitlines() if not l.startswith(drop)]
    assert keep(body) == keep(expected)


@pytest.mark.gpu
@need_ref
@need_amd
@pytest.mark.parametrize("fmt", FORMATS)
def test_shim_matches_reference_cli(bam_pairs, fmt):
    for d in bam_pairs:
        for opts in OPTSETS:
            args = ["-F", fmt] + opts + ["-f", "ref.fa", "tumor.bam", "normal.bam"]
            rc_r, ref, err_r = run(REF_CLI, args, d)
            env = dict(os.environ, SS_SHIM_BATCH="777")          # several flushes per run
            rc_a, amd, err_a = run(AMD_CLI, args, d, env=env)
            assert rc_r == 0 and rc_a == 0, (err_r, err_a)
            assert strip_volatile(amd) == strip_volatile(ref), (d, fmt, opts)
