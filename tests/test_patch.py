"""The libyara call-site patch (integration/libyara-block-scanner.patch) is a
real patch: it applies cleanly to the reference tree (CPU; skipped where the
reference is absent, e.g. on the GPU box, which runs the patched build)."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

REF = os.environ.get("YARA_REFERENCE", "/root/reference")
PATCH = os.path.join(REPO, "integration", "libyara-block-scanner.patch")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "libyara")), reason="no reference tree")
def test_patch_applies_to_reference(tmp_path):
    for rel in ("libyara/scanner.c", "libyara/include/yara/types.h",
                "libyara/include/yara/scanner.h"):
        dst = tmp_path / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(REF, rel), str(dst))
        os.chmod(str(dst), 0o644)
    p = subprocess.run(["patch", "-p1", "--dry-run", "-d", str(tmp_path), "-i", PATCH],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "FAILED" not in p.stdout and "fuzz" not in p.stdout


def test_patch_touches_only_the_call_site_and_api():
    text = open(PATCH).read()
    files = [l.split()[1] for l in text.splitlines() if l.startswith("+++ ")]
    assert files == ["b/libyara/include/yara/types.h", "b/libyara/include/yara/scanner.h",
                     "b/libyara/scanner.c"]
    added = [l for l in text.splitlines() if l.startswith("+") and not l.startswith("+++")]
    assert len(added) < 80
    assert any("block_scanner->scan_block" in l for l in added)
