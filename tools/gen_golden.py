"""Generate golden parity fixtures by running the REFERENCE simulator.

The reference (read-only, /root/reference) needs vLLM, which is not installed;
we put a stub ``vllm`` package on sys.path whose ``LLM.generate`` answers every
prompt with ``engine/fake.py:scripted_text`` -- the same function this
framework's ``fake`` backend uses.  For each configuration we record the exact
formatted prompts the reference sent (in order), its engine-call count, and
its results JSON.  tests/test_parity_reference.py replays the same seeds
through our simulator and diffs everything.

Usage: python tools/gen_golden.py [--reference /root/reference] [--out tests/golden]
"""
import argparse
import importlib.util
import json
import os
import random
import shutil
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

def _r(agent, rnd, phase, tries, mode):
    return {"agent": agent, "round": rnd, "phase": phase, "tries": tries, "mode": mode}


# Retry-ladder failure paths (reference main.py:293-352 decide, :376-478 vote,
# vllm_agent.py:445-448 engine exception), injected deterministically
# (engine/fake.py FaultInjector) into the SAME scripted engine on both sides.
FAULTS_H8B2 = [
    _r("agent_1", 1, "decide", [1, 2], "invalid_json"),        # <=30 % -> sequential, succeeds on its 2nd try
    _r("agent_4", 1, "decide", [1, 2, 3, 4], "invalid_json"),  # sequential: all 3 fail -> abstains
    *[_r(f"agent_{i}", 2, "decide", [1], "short") for i in (0, 2, 5, 7)],  # 40 % -> re-batch
    _r("agent_9", 3, "decide", [1, 2], "short"),               # batch-invalid, sequential-valid answer
    _r("agent_3", 1, "vote", [1, 2, 3, 4], "invalid_json"),    # sequential vote: all fail
    *[_r(f"agent_{i}", 2, "vote", [1], "short") for i in (1, 6, 8, 9)],  # 40 % -> re-batch
    _r("agent_2", 3, "vote", [1], "short"),                    # <=30 % -> sequential, succeeds
    *[_r(f"agent_{i}", 4, "vote", [1, 2, 3], "invalid_json") for i in (0, 3, 5, 8)],  # 40 % x3 -> default continue
]
FAULTS_H4B0 = [
    _r("agent_0", 1, "decide", [1], "exception"),              # engine raises -> {"error"} for all -> re-batch
    _r("agent_1", 1, "vote", [1, 2, 3], "exception"),          # every batched vote attempt raises -> default continue
    _r("agent_2", 2, "decide", [1, 2, 3], "exception"),        # every decide attempt raises -> all abstain
]

CONFIGS = [
    # name, honest, byzantine, max_rounds, seed, awareness, value_range[, fault plan]
    ("h4b0", 4, 0, 5, 11, "may_exist", (0, 50)),
    ("h4b1", 4, 1, 6, 5, "may_exist", (0, 50)),
    ("h8b2", 8, 2, 4, 7, "may_exist", (0, 50)),
    ("h5b0_none", 5, 0, 4, 3, "none_exist", (10, 20)),
    ("h3b2", 3, 2, 5, 2, "may_exist", (0, 9)),
    ("h8b2_faults", 8, 2, 4, 7, "may_exist", (0, 50), FAULTS_H8B2),
    ("h4b0_exceptions", 4, 0, 6, 11, "may_exist", (0, 50), FAULTS_H4B0),
]


def load_fake():
    path = os.path.join(REPO, "byzantine_consensus_llm_agents_amd", "engine", "fake.py")
    spec = importlib.util.spec_from_file_location("_bcg_fake", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def install_stub_vllm(log, faults=None):
    fake = load_fake()
    injector = fake.FaultInjector(faults) if faults else None
    vllm = types.ModuleType("vllm")
    sp = types.ModuleType("vllm.sampling_params")

    class GuidedDecodingParams:
        def __init__(self, json=None, **kw):
            self.json = json

    class SamplingParams:
        def __init__(self, temperature=1.0, top_p=1.0, max_tokens=16, guided_decoding=None, **kw):
            self.temperature, self.max_tokens, self.guided_decoding = temperature, max_tokens, guided_decoding

    class _Out:
        def __init__(self, text):
            self.outputs = [types.SimpleNamespace(text=text)]

    class LLM:
        def __init__(self, **kw):
            self.kw = kw

        def generate(self, prompts, params):
            schema = params.guided_decoding.json if params.guided_decoding else None
            log.append({"n": len(prompts), "temperature": params.temperature, "max_tokens": params.max_tokens})
            for p in prompts:
                log[-1].setdefault("prompts", []).append(p)
                log[-1].setdefault("schemas", []).append(schema)
            if injector is not None:
                return [_Out(t) for t in injector.answer_batch(prompts, [schema] * len(prompts), 0)]
            return [_Out(fake.scripted_text(p, schema, 0)) for p in prompts]

    vllm.LLM, vllm.SamplingParams = LLM, SamplingParams
    sp.GuidedDecodingParams = GuidedDecodingParams
    vllm.sampling_params = sp
    sys.modules["vllm"] = vllm
    sys.modules["vllm.sampling_params"] = sp


def run_reference(ref_dir, name, honest, byz, rounds, seed, awareness, vr, faults=None):
    log = []
    install_stub_vllm(log, faults)
    src = os.path.join(ref_dir, "byzantine_consensus_game")
    for m in ["config", "main", "byzantine_consensus", "a2a_sim", "agent_network",
              "communication_protocol", "protocol_factory", "bcg_agents", "vllm_agent"]:
        sys.modules.pop(m, None)
    sys.path.insert(0, src)
    cwd = os.getcwd()
    work = tempfile.mkdtemp()
    os.chdir(work)
    try:
        import config as rcfg
        import main as rmain
        rcfg.BCG_CONFIG["value_range"] = vr
        random.seed(seed)
        sim = rmain.BCGSimulation(num_honest=honest, num_byzantine=byz, config={
            "max_rounds": rounds, "consensus_threshold": 66.0, "value_range": vr,
            "verbose": False, "byzantine_awareness": awareness})
        # reference bug: display_results() formats byzantine_infiltration=None with
        # :.1f when 0 Byzantine agents reach consensus (main.py:726) and crashes
        # before saving; the golden run bypasses the display so the results
        # still get written.  Our simulator prints "n/a" instead (documented).
        orig_display = sim.display_results

        def safe_display():
            try:
                orig_display()
            except TypeError:
                pass
        sim.display_results = safe_display
        sim.run()
        with open(os.path.join("results", "json", "run_001.json")) as fh:
            results = json.load(fh)
        with open(os.path.join("results", "metrics", "run_001.csv")) as fh:
            csv_text = fh.read()
        with open(os.path.join("results", "logs", "run_001_log.txt")) as fh:
            log_text = fh.read() if faults else None
    finally:
        os.chdir(cwd)
        sys.path.remove(src)
        shutil.rmtree(work, ignore_errors=True)
        rcfg.BCG_CONFIG["value_range"] = (0, 50)
    results.pop("timestamp", None)
    results["metrics"].pop("timestamp", None)
    csv_lines = csv_text.splitlines()
    return {"name": name, "honest": honest, "byzantine": byz, "rounds": rounds, "seed": seed,
            "awareness": awareness, "value_range": list(vr), "engine_calls": log,
            "results": results, "csv_header": csv_lines[0], "faults": faults or [], "log": log_text}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden"))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    for cfg in CONFIGS:
        rec = run_reference(args.reference, *cfg)
        path = os.path.join(args.out, f"ref_{cfg[0]}.json")
        with open(path, "w") as fh:
            json.dump(rec, fh, indent=1, sort_keys=True)
        calls = rec["engine_calls"]
        print(f"{path}: {len(calls)} engine calls, {sum(c['n'] for c in calls)} prompts, "
              f"outcome={rec['results']['statistics']['consensus_outcome']}")


if __name__ == "__main__":
    main()
