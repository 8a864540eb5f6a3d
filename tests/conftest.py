import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


import pytest  # noqa: E402


class KnobPatch:
    """monkeypatch's setenv / delenv for the switches the tests flip between launches: the library's A/B knobs go
    through vp_set_knob (the library reads the environment once, at load), the Python-side switches (e.g.
    VP_NO_QKV_FUSION, read once at import) through attention_processor.set_switch; everything is restored at
    teardown."""

    def __init__(self, mp):
        self.mp = mp
        self.saved = []

    def _lib(self, name, value):
        from videopainter_amd import _native as N
        from videopainter_amd import attention_processor as AP
        from videopainter_amd import kernels as K
        if name in N.KNOBS:
            self.saved.append((name, K.set_knob(name, value)))
        elif name in AP.SWITCHES:
            self.saved.append((name, AP.set_switch(name, value)))

    def setenv(self, name, value):
        self.mp.setenv(name, value)
        self._lib(name, value)

    def delenv(self, name, raising=True):
        self.mp.delenv(name, raising=raising)
        self._lib(name, None)

    def __getattr__(self, attr):  # setattr, delitem, ...: plain monkeypatch
        return getattr(self.mp, attr)

    def undo(self):
        from videopainter_amd import attention_processor as AP
        from videopainter_amd import kernels as K
        for name, prev in reversed(self.saved):
            if name in AP.SWITCHES:
                AP.set_switch(name, prev)
            else:
                K.set_knob(name, prev)
        self.saved.clear()


@pytest.fixture
def knobs(monkeypatch):
    kp = KnobPatch(monkeypatch)
    yield kp
    kp.undo()
