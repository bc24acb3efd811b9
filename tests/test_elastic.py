"""Elastic recovery from a lost node (CPU, gloo; SURVEY §5 "Crash/OFFLINE").

A 3-rank GPT-2 pipeline runs under ``runtime/elastic.ElasticSupervisor``; rank 2 is SIGKILLed after
optimizer step 5, or hangs there with its heartbeat stopped (``TDL_FAULT_INJECT``, generation 0
only).  The survivors' heartbeat watchdogs mark
it OFFLINE and abort (code 17) instead of hanging in the next collective; the supervisor relaunches
on the two survivors with ``--resume latest``: the newest complete checkpoint (step 4) is re-planned
over 2 ranks and training continues at the saved batch to the end of the epoch."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stats(log_path):
    text = open(log_path).read()
    i = text.rfind("\n{\n")
    assert i >= 0, text[-3000:]
    return json.loads(text[i + 1:text.rfind("}") + 1])


def test_blame_by_severity():
    from trustworthy_dl.runtime.elastic import ABORT_CODE, blame
    assert blame({1: -6, 2: -9}) == [2]            # SIGABRT of the comm library is collateral
    assert blame({0: 1, 2: -11}) == [2]
    assert blame({0: ABORT_CODE, 1: 1}) == [1]     # an ordinary error exit outranks a heartbeat abort
    assert blame({0: ABORT_CODE, 1: -6}) == [1]
    assert blame({0: ABORT_CODE}) == []


def test_checkpoint_faults_parse():
    from trustworthy_dl.runtime import faults
    fs = faults.parse("crash:rank=2:step=5;hang:rank=0:step=9:gen=1")
    assert fs == [{"kind": "crash", "rank": 2, "step": 5, "gen": 0}, {"kind": "hang", "rank": 0, "step": 9, "gen": 1}]
    with pytest.raises(ValueError):
        faults.parse("explode:rank=0")


@pytest.mark.slow
@pytest.mark.timeout(300)
@pytest.mark.parametrize("fault,victim", [("crash", 2), ("hang", 2), ("crash", 1)])
def test_elastic_shrink_and_resume(tmp_path, fault, victim):
    from trustworthy_dl.runtime.elastic import ElasticSupervisor
    ck = tmp_path / "ck"
    logs = tmp_path / "logs"
    args = ["--model", "gpt2-tiny", "--dataset", "markov", "--device", "cpu", "--dtype", "fp32", "--seq-len", "32",
            "--batch-size", "8", "--micro-batches", "4", "--epochs", "1", "--batches-per-epoch", "12", "--lr", "1e-3",
            "--heartbeat", "0.3", "--heartbeat-timeout", "4", "--checkpoint-interval", "2",
            "--checkpoint-dir", str(ck)]
    env = dict(os.environ, TDL_FAULT_INJECT=f"{fault}:rank={victim}:step=5", OMP_NUM_THREADS="2",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    sup = ElasticSupervisor(args, nproc=3, min_nproc=2, max_restarts=2, grace_s=20, timeout_s=240, env=env,
                            python=sys.executable, log_dir=str(logs))
    res = sup.run()
    g0, g1 = res["generations"][0], res["generations"][-1]
    assert res["ok"], res
    assert len(res["generations"]) == 2, res
    assert g0["lost"] == [victim], res
    assert g0["exit_codes"][victim] < 0              # killed by a signal (SIGKILL crash / our SIGTERM)
    # survivors never finished: under gloo the closed connection raises in the next collective
    # (exit 1) before the heartbeat timeout; under RCCL they would hang and abort with ABORT_CODE
    survivors = [r for r in range(3) if r != victim]
    assert all(g0["exit_codes"][r] not in (0, None) for r in survivors), res
    assert g1["world"] == 2 and res["final_world"] == 2
    assert g1["node_ids"] == survivors, res         # new ranks carry the survivors' physical identity
    st = _stats(logs / "gen1.rank0.log")
    assert st["global_step"] == 12, st              # resumed at the step-4 checkpoint, trained batches 4..11
    assert st["training_state"] == "completed"
    assert st["reassignment_count"] >= 1            # the resume re-plan is recorded
    assert len(st["plan"].split(";")) == 2 or st["plan"].count("@rank") == 2, st["plan"]


def test_restart_resumes_latest_not_user_path():
    """a user --resume <path> must not pin every later generation to that path"""
    from trustworthy_dl.runtime.elastic import ElasticSupervisor
    sup = ElasticSupervisor(["--model", "gpt2-tiny", "--resume", "/old/ck.pt", "--epochs", "1"], nproc=2,
                            devices=["0", "1"])
    assert sup._cmd(0)[-4:] == ["--resume", "/old/ck.pt", "--epochs", "1", "--abort-on-offline"][-4:]
    c1 = sup._cmd(1)
    assert "/old/ck.pt" not in c1 and c1[-2:] == ["--resume", "latest"]
    sup2 = ElasticSupervisor(["--resume=/old/ck.pt"], nproc=2, devices=["0", "1"])
    assert "--resume=/old/ck.pt" not in sup2._cmd(2)


def test_default_devices_follow_visible_list():
    """without --devices the lost rank's GPU must be the one dropped"""
    from trustworthy_dl.runtime.elastic import default_devices
    assert default_devices(3, {"HIP_VISIBLE_DEVICES": "4,5,6,7"}) == ["4", "5", "6"]
    assert default_devices(2, {"ROCR_VISIBLE_DEVICES": "1,3"}) == ["1", "3"]


def test_node_ids_env_roundtrip(monkeypatch):
    from trustworthy_dl.runtime.elastic import node_ids_from_env
    monkeypatch.setenv("TDL_ELASTIC_NODE_IDS", "0,2,3")
    assert node_ids_from_env(3) == [0, 2, 3]
    assert node_ids_from_env(2) == [0, 1]           # malformed for this world: identity
    monkeypatch.delenv("TDL_ELASTIC_NODE_IDS")
    assert node_ids_from_env(2) == [0, 1]


def test_trust_follows_physical_node_after_losing_rank1(monkeypatch):
    """after losing rank 1 of 3 the survivors are renumbered 0, 1; the compromised node 1's
    record must NOT land on new rank 1 (= physical node 2), and node 2's record must not be dropped."""
    import torch
    from trustworthy_dl.core.trust_manager import NodeStatus, TrustManager
    from trustworthy_dl.utils.checkpoint import _resize_trust
    old = TrustManager(num_nodes=3)
    old.mark_compromised(1, "gradient_poisoning")
    old.update_trust_score(2, 0.4, 0.6)
    saved = {"trust_manager": old.state_dict(), "node_ids": [0, 1, 2], "excluded": [1],
             "device_trust": {"values": torch.tensor([0.9, 0.1, 0.55]), "counts": torch.tensor([5, 5, 5]),
                              "status": torch.tensor([0, 2, 1])}}

    class _Eng:
        excluded = []
        st = {"values": torch.ones(2), "counts": torch.zeros(2, dtype=torch.long),
              "status": torch.zeros(2, dtype=torch.long)}

        def trust_state(self):
            return {k: v.clone() for k, v in self.st.items()}

        def load_trust_state(self, sd, partial=False):
            self.st = sd

    class _Tr:
        trust_manager = TrustManager(num_nodes=2)
        engine = _Eng()

    tr = _Tr()
    monkeypatch.setenv("TDL_ELASTIC_NODE_IDS", "0,2")
    _resize_trust(tr, saved, 2)
    tm = tr.trust_manager
    assert tm.get_node_status(1) != NodeStatus.COMPROMISED            # new rank 1 is physical node 2
    assert abs(tm.get_trust_score(1) - old.get_trust_score(2)) < 1e-9
    assert abs(tm.get_trust_score(0) - old.get_trust_score(0)) < 1e-9
    assert tr.engine.st["values"].tolist() == [0.8999999761581421, 0.550000011920929]
    assert tr.engine.excluded == []                                    # excluded node 1 is gone
    # losing rank 0 instead: node 1 (compromised) becomes new rank 0 and stays compromised + excluded
    tr2 = _Tr()
    tr2.trust_manager = TrustManager(num_nodes=2)
    tr2.engine = _Eng()
    monkeypatch.setenv("TDL_ELASTIC_NODE_IDS", "1,2")
    _resize_trust(tr2, saved, 2)
    assert tr2.trust_manager.get_node_status(0) == NodeStatus.COMPROMISED
    assert tr2.engine.excluded == [0]


def test_resume_plan_leaves_excluded_physical_node_out(monkeypatch):
    """saved plan [0, 2] with node 1 excluded, then rank 0 is lost.  The survivors are
    physical nodes 1, 2 (new ranks 0, 1): the saved stage of node 2 runs on new rank 1, node 0's
    stage is gone, so the plan is re-planned — and never onto new rank 0 (compromised node 1)."""
    import torch
    from trustworthy_dl.utils.checkpoint import resume_plan_ranks
    ck = {"node_ids": [0, 1, 2], "excluded": [1], "device_trust": {"values": torch.ones(3)}}
    monkeypatch.setenv("TDL_ELASTIC_NODE_IDS", "1,2")
    moved, live_ex = resume_plan_ranks(ck, [0, 2], live=2, pp=2)
    assert moved is None and live_ex == [0]
    live = [r for r in range(2) if r not in live_ex]
    assert live == [1]
    # losing node 1 (the excluded one) instead: the saved plan is hostable, its ranks translated
    monkeypatch.setenv("TDL_ELASTIC_NODE_IDS", "0,2")
    moved, live_ex = resume_plan_ranks(ck, [0, 2], live=2, pp=2)
    assert moved == [0, 1] and live_ex == []
    # a plan that put a stage on the excluded node is never adopted
    monkeypatch.setenv("TDL_ELASTIC_NODE_IDS", "0,1,2")
    moved, live_ex = resume_plan_ranks(ck, [0, 1], live=3, pp=3)
    assert moved is None and live_ex == [1]
