"""Independent predicts on several streams at once (-m gpu): the lazily built caches a
predict fills (packed weights, a snapshot's relation-type edge order, parameter-only states)
are read by whichever stream asks next, so each is published (regcn_amd._lib.publish) before
it is cached.  A fresh model and fresh snapshot graphs, three streams started together with
no warm-up: every predict must equal the reference golden, as a sequential one does."""
import numpy as np
import pytest
import torch

from gpu_helpers import assert_close, build_hyperbolic_model

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("tag,layers", [("uvrgcn_roth", False), ("uvrgcn_roth", True), ("lgcn_roth", False)])
def test_concurrent_predicts_on_streams(golden, tag, layers):
    z = golden("model_%s.npz" % tag)
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, DEV)
    m.use_phases = not layers  # both encoder launch shapes (per-layer: the config-5 path)
    test = torch.from_numpy(z["test"]).to(DEV)
    torch.cuda.synchronize()
    main = torch.cuda.current_stream(DEV)
    streams = [torch.cuda.Stream(DEV) for _ in range(3)]
    outs = []
    with torch.no_grad():
        for st in streams:
            st.wait_stream(main)
            with torch.cuda.stream(st):
                outs.append(m.predict(glist, R, None, test, True))
        for st in streams:
            main.wait_stream(st)
        torch.cuda.synchronize()
    for all_tr, score, score_rel in outs:
        np.testing.assert_array_equal(all_tr.cpu().numpy(), z["all_triples"])
        assert_close(score, z["score"], what="entity score")
        assert_close(score_rel, z["score_rel"], what="relation score")
    # and bit for bit the same across the streams (no atomics)
    for o in outs[1:]:
        assert torch.equal(o[1], outs[0][1]) and torch.equal(o[2], outs[0][2])
