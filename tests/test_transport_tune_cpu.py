"""parallel/transport_tune.py: the world > 1 transport configuration chosen from injected link
times (bench.py ``--transport-tune`` measures them on the live node before the model is built)."""
import pytest

from torch_distributed_sandbox_amd.parallel import transport_tune as TT

M = TT.StepModel(local_ms=2.0, exchange_ms=0.6, split_ms={0: 0.0, 32: 0.1, 64: 0.3}, window_ms=2.4,
                 interference=0.5)


def _measure(table):
    def measure(cfg):
        v = table[(cfg.reserve_cus, cfg.max_ctas)]
        if isinstance(v, Exception):
            raise v
        return v

    return measure


def test_predict_matches_the_model():
    # 32-CU split, gathers hidden in the window: local + exchange + split
    assert TT.predict_ms(TT.TransportConfig(32, 32), 2.0, M) == pytest.approx(2.7)
    # link time past the window is exposed
    assert TT.predict_ms(TT.TransportConfig(32, 32), 3.4, M) == pytest.approx(3.7)
    # no split: the collective's workgroups collide with the persistent kernels
    assert TT.predict_ms(TT.TransportConfig(0, 0), 2.0, M) == pytest.approx(2.6 + 1.0)
    # an unmeasured split is interpolated
    assert TT.predict_ms(TT.TransportConfig(48, 48), 1.0, M) == pytest.approx(2.6 + 0.2)


def test_fast_links_keep_the_small_split():
    # every config hides its gathers: the cheapest split wins
    r = TT.choose(_measure({(32, 32): 1.5, (64, 64): 1.0, (0, 0): 1.2}), M)
    assert r["chosen"] == {"reserve_cus": 32, "max_ctas": 32}
    assert [c["predicted_step_ms"] for c in r["candidates"]] == [2.7, 2.9, pytest.approx(3.2)]


def test_cta_bound_links_take_the_bigger_split():
    # 32 CTAs cannot drive the links: 4.0 ms of gathers, 64 CTAs 2.5 ms
    r = TT.choose(_measure({(32, 32): 4.0, (64, 64): 2.5, (0, 0): 2.3}), M)
    assert r["chosen"] == {"reserve_cus": 64, "max_ctas": 64}
    assert r["predicted_step_ms"] == pytest.approx(2.0 + 0.6 + 0.3 + 0.1)


def test_unsplit_wins_when_collectives_are_tiny():
    r = TT.choose(_measure({(32, 32): 0.05, (64, 64): 0.05, (0, 0): 0.05}), M)
    assert r["chosen"] == {"reserve_cus": 0, "max_ctas": 0}


def test_failed_candidate_is_skipped_and_recorded():
    r = TT.choose(_measure({(32, 32): RuntimeError("maxCTAs rejected"), (64, 64): 2.0, (0, 0): 5.0}), M)
    assert r["chosen"] == {"reserve_cus": 64, "max_ctas": 64}
    assert "maxCTAs rejected" in r["candidates"][0]["error"]
    assert "predicted_step_ms" not in r["candidates"][0]


def test_nothing_measurable_chooses_nothing():
    r = TT.choose(_measure({(32, 32): OSError("x"), (64, 64): OSError("y"), (0, 0): OSError("z")}), M)
    assert r["chosen"] is None and r["predicted_step_ms"] is None
    assert len(r["candidates"]) == 3


@pytest.mark.parametrize("world,path", [(2, "activations"), (4, "activations"), (8, "sharded")])
def test_probe_moves_what_the_step_moves(world, path):
    K = 32 * 750 ** 2
    p, colls = TT.step_collectives(world, 5, 10, K)
    assert p == path
    if path == "activations":
        assert colls[0] == ("all_gather", int(5 * K * 4 * 0.6))
    else:
        assert colls[1] == ("sendrecv", 10 * (-(-K // world)) * 4)
