"""The fake hive lives in the package (chiaswarm_amd/hive/fake.py) so
``bench.py --through-supervisor`` can drive it too."""
from chiaswarm_amd.hive.fake import FakeHive, dumps  # noqa: F401
