"""Mid-size goldens of the benchmarked configurations (tests/golden/midsize.json,
made offline by the CPU oracle with tests/golden/make_golden_mid.py, which
takes tens of minutes per case): the GPU engine must reproduce every counter
and every readback digest bit for bit at sizes where the production kernel
instantiations, arena sizes and LDS tables are those of the 1M-peer runs.

  c4mid  config4 (64 topics x 256 slots, k = 32, Eth2 scoring) at 30,000 peers
  c3mid  config3 (1 topic x 10048 slots) at 10,000 peers, 8 rounds: the
         MaxIHaveLength cut mode of config3's steady state"""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden_mid  # noqa: E402
from make_golden import digest  # noqa: E402

PATH = os.path.join(HERE, "golden", "midsize.json")
GOLDEN = json.load(open(PATH)) if os.path.exists(PATH) else {}

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_gpu_reproduces_midsize_golden(name):
    from pubsub_amd import PRODUCT_LIB
    got = digest(make_golden_mid.run(PRODUCT_LIB, name))
    want = GOLDEN[name]
    assert got["counters"] == want["counters"]
    bad = sorted(k for k in want if got.get(k) != want[k])
    assert not bad, f"{name}: readbacks differ from the oracle's: {bad}"
