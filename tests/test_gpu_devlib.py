"""The devlib tests against the dev library (make dev: kaolin/_lib/dev/libkaolin_hip.so, KL_DEV=1).

The product library carries no dev controls (no process-global mutable state; the
measured dead ends compiled out).  The tests that switch between the product path and a measured
alternative, or force a fallback branch (pair-buffer overflow, list caps, the hit-list march's
fallback), need them: they run here, in one child pytest process on the dev build (KAOLIN_HIP_LIB;
KAOLIN_NO_EXT=1 so that the compiled autograd node does not load the product library beside it),
under its own time limit.  In this process they skip the parts that need the dev library.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
DEV_LIB = os.path.join(ROOT, 'kaolin-windows_amd', 'kaolin', '_lib', 'dev', 'libkaolin_hip.so')


def test_devlib_tests_on_the_dev_build():
    if os.environ.get('KAOLIN_HIP_LIB'):
        pytest.skip('already running on a chosen library')
    assert os.path.exists(DEV_LIB), 'dev library missing: make -C kaolin-windows_amd/csrc dev'
    env = dict(os.environ, KAOLIN_HIP_LIB=DEV_LIB, KAOLIN_NO_EXT='1')
    r = subprocess.run([sys.executable, '-u', '-m', 'pytest', HERE, '-m', 'gpu and devlib', '-q', '-x', '-rs',
                        '-p', 'no:cacheprovider', '--timeout', '120', '--timeout-method', 'thread'],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert ' passed' in r.stdout and 'needs the dev library' not in r.stdout, tail
