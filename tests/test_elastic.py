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


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fault", ["crash", "hang"])
def test_elastic_shrink_and_resume(tmp_path, fault):
    from trustworthy_dl.runtime.elastic import ElasticSupervisor
    ck = tmp_path / "ck"
    logs = tmp_path / "logs"
    args = ["--model", "gpt2-tiny", "--dataset", "markov", "--device", "cpu", "--dtype", "fp32", "--seq-len", "32",
            "--batch-size", "8", "--micro-batches", "4", "--epochs", "1", "--batches-per-epoch", "12", "--lr", "1e-3",
            "--heartbeat", "0.3", "--heartbeat-timeout", "4", "--checkpoint-interval", "2",
            "--checkpoint-dir", str(ck)]
    env = dict(os.environ, TDL_FAULT_INJECT=f"{fault}:rank=2:step=5", OMP_NUM_THREADS="2",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    sup = ElasticSupervisor(args, nproc=3, min_nproc=2, max_restarts=2, grace_s=20, timeout_s=240, env=env,
                            python=sys.executable, log_dir=str(logs))
    res = sup.run()
    g0, g1 = res["generations"][0], res["generations"][-1]
    assert res["ok"], res
    assert len(res["generations"]) == 2, res
    assert g0["lost"] == [2], res
    assert g0["exit_codes"][2] < 0                   # killed by a signal (SIGKILL crash / our SIGTERM)
    # survivors never finished: under gloo the closed connection raises in the next collective
    # (exit 1) before the heartbeat timeout; under RCCL they would hang and abort with ABORT_CODE
    assert all(g0["exit_codes"][r] not in (0, None) for r in (0, 1)), res
    assert g1["world"] == 2 and res["final_world"] == 2
    st = _stats(logs / "gen1.rank0.log")
    assert st["global_step"] == 12, st              # resumed at the step-4 checkpoint, trained batches 4..11
    assert st["training_state"] == "completed"
    assert st["reassignment_count"] >= 1            # the resume re-plan is recorded
    assert len(st["plan"].split(";")) == 2 or st["plan"].count("@rank") == 2, st["plan"]
