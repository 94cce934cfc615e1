"""The example scripts run end to end on CPU (tiny random-init model / stub server)."""
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.timeout(600)
def test_agent_example_forced_tool_call():
    out = subprocess.run([sys.executable, str(ROOT / "examples/agent.py"), "--model", "tiny-llama", "--device", "cpu",
                          "--max-iterations", "2", "--prompt-sections", "intro,core_tools", "--tool-choice",
                          '{"type":"function","function":{"name":"get_weather"}}'],
                         capture_output=True, text=True, timeout=600,
                         # two intra-op threads: under pytest -n the runs share the CPUs, and 8-thread OpenMP pools
                         # oversubscribed 4x spend their time in barriers (15 s alone, > 150 s with 4 at once)
                         env={"OMP_NUM_THREADS": "2", **os.environ, "KAFKA_WEATHER_MODE": "offline"})
    assert out.returncode == 0, out.stderr[-2000:]
    assert "[tool call] get_weather" in out.stdout and "[tool result] Weather in" in out.stdout
    assert "[done]" in out.stdout


@pytest.mark.timeout(300)
def test_client_example_against_stub_server():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, KAFKA_LLM_BACKEND="stub", KAFKA_SANDBOX="none", LOCAL_DB_PATH=":memory:",
               PYTHONPATH=str(ROOT))
    srv = subprocess.Popen([sys.executable, "-m", "kafka_llm_service_amd.server", "--host", "127.0.0.1", "--port",
                            str(port)], env=env)
    try:
        import httpx

        for _ in range(100):
            try:
                if httpx.get(f"http://127.0.0.1:{port}/health").status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.2)
        out = subprocess.run([sys.executable, str(ROOT / "examples/client.py"), "--url", f"http://127.0.0.1:{port}"],
                             capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr[-2000:]
        assert "history: ['user', 'assistant', 'user', 'assistant']" in out.stdout and "[usage]" in out.stdout
    finally:
        srv.terminate()
        srv.wait(timeout=30)
