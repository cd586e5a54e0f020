"""utils/host_sampler.py: the engine thread's busy frame and the running-thread census."""
import threading
import time

from byzantine_consensus_llm_agents_amd.utils.host_sampler import HostSampler


def test_host_sampler_finds_the_busy_engine_frame():
    stop = time.time() + 0.6

    def spin():  # busy, but yielding the GIL now and then (as a thread in C calls does)
        while time.time() < stop:
            t = time.time()
            while time.time() - t < 0.004:
                sum(range(200))
            time.sleep(0.0002)

    th = threading.Thread(target=spin, name="bcg-engine-test")
    s = HostSampler(interval=0.01).start()
    th.start()
    th.join()
    out = s.stop()
    assert out["samples"] >= 3
    assert out["engine_innermost"] and "spin" in out["engine_innermost"][0][0]
    running = dict(out["running_threads"])
    # (a Python thread is seen R only between GIL hand-offs -- the sampler needs the GIL to
    # sample; native pools are seen exactly)
    assert "bcg-engine-test" in running or out["thread_counts"].get("bcg-engine-test") == 1
    assert out["thread_counts"].get("bcg-engine-test") == 1
