"""Cached-key strict verdicts at every launch size the verify dispatch distinguishes, on the golden
adversarial cases (non-canonical / undecodable / small-order R and A, x = 0 with the sign bit set,
wrong sign, bad S, ...):

  <= 16,384 signatures   k_verify_split (8 lanes per signature) + k_finish<true> (one inversion per lane;
                         variable-time for <= 8 signatures)
  > 16,384               k_verify + k_finish

Each must reproduce the oracle's verify_strict verdict (tests/golden adversarial_strict) bit for bit.
"""
import pytest

pytestmark = pytest.mark.gpu

ZSEED = bytes(range(32))


@pytest.fixture(scope="module")
def adv(golden):
    from narwhal_amd import _lib
    cases = golden["adversarial_strict"]
    eng = _lib.Engine(device=0)
    pks = [bytes.fromhex(c["pk"]) for c in cases]
    slots = eng.committee_load(pks, [1] * len(pks))
    yield eng, cases, slots
    eng.close()


def _run(eng, cases, slots, n):
    idx = [i % len(cases) for i in range(n)]
    msgs = [bytes.fromhex(cases[k]["msg"]) for k in idx]
    sigs = [bytes.fromhex(cases[k]["sig"]) for k in idx]
    # one batch per signature: every verdict is the strict one
    _, sig_ok = eng.verify_batches([(i, 1) for i in range(n)], msgs, [slots[k] for k in idx], sigs, ZSEED)
    return sig_ok


def test_each_case_alone(adv):
    eng, cases, slots = adv
    for c, s in zip(cases, slots):
        _, ok = eng.verify_batches([(0, 1)], [bytes.fromhex(c["msg"])], [s], [bytes.fromhex(c["sig"])], ZSEED)
        assert ok == [c["strict"]], c["name"]


@pytest.mark.parametrize("target", [8, 9, 67, 2048, 16384, 16385, 20000])
def test_launch_sizes(adv, target):
    eng, cases, slots = adv
    got = _run(eng, cases, slots, target)
    bad = sorted({cases[i % len(cases)]["name"] for i in range(target) if got[i] != cases[i % len(cases)]["strict"]})
    assert not bad, (target, bad)
