"""GPU: the reference's transaction-level unit tests (tests/golden/reference_test_scenarios.json)
through the HIP path: writes on the host write path, then each read / scan published
(stage_sync) and answered by the device probe / scan kernels; every outcome the reference
tests assert must hold (Lookup-Old through the version chain, aborted updates and inserts,
in-flight copies, BTreeTest Update / Upsert)."""
import pytest

import scenarios as S

pytestmark = pytest.mark.gpu
SCEN = S.load()


@pytest.mark.parametrize("sc", SCEN, ids=[s["name"] for s in SCEN])
def test_device_meets_reference_assertions(gpu, sc):
    assert S.run(sc, S.DeviceBackend) == []
