"""A/B probe: the late schedule with ONE forced Newton–Schulz step (sbr_device.LATE_NS_ITERS = 1)
for the bench (argv: bench args) or pytest (argv[1] == 'pytest')."""
import os
import sys

sys.path.insert(0, os.getcwd())
import evoxmi.ops.sbr_device as sd  # noqa: E402

sd.LATE_NS_ITERS = int(os.environ.get("NS_LATE", str(sd.LATE_NS_ITERS)))
sd.LATE_FULL_SLOTS = int(os.environ.get("LATE_FULL", str(sd.LATE_FULL_SLOTS)))
sd.DEVICE_CFG["ns_iters"] = int(os.environ.get("NS_WARM", str(sd.DEVICE_CFG["ns_iters"])))
if len(sys.argv) > 1 and sys.argv[1] == "pytest":
    import pytest

    sys.exit(pytest.main(sys.argv[2:]))
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
