"""``python -m kafka_llm_service_amd.server`` — run the API server (the reference's ``python server.py``, port 8081 by
default, /root/reference/server.py:627-631). Configuration comes from the environment (``ServerConfig.from_env``:
KAFKA_LLM_BACKEND, KAFKA_MODEL, KAFKA_DP, KAFKA_TP, LOCAL_DB_PATH, KAFKA_SANDBOX, LOCAL_SANDBOX_URL, ...)."""
from __future__ import annotations

import argparse
import os


# CLI flag -> environment variable read by ServerConfig.from_env (flags win over the environment)
FLAGS = {"backend": "KAFKA_LLM_BACKEND", "model": "KAFKA_MODEL", "weights": "KAFKA_WEIGHTS", "dp": "KAFKA_DP",
         "tp": "KAFKA_TP", "max_model_len": "KAFKA_MAX_MODEL_LEN", "db": "KAFKA_DB", "db_path": "LOCAL_DB_PATH",
         "sandbox": "KAFKA_SANDBOX", "sandbox_url": "LOCAL_SANDBOX_URL", "tool_choice": "KAFKA_TOOL_CHOICE",
         "prompt_sections": "KAFKA_PROMPT_SECTIONS", "served_model_name": "DEFAULT_MODEL",
         "kv_dtype": "KAFKA_KV_DTYPE"}


def main() -> None:
    ap = argparse.ArgumentParser(description="kafka-llm-service-amd API server")
    ap.add_argument("--host", default=os.environ.get("HOST", "0.0.0.0"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("PORT", "8081")))
    ap.add_argument("--log-level", default="warning", help="uvicorn access/error log level")
    ap.add_argument("--log-json", action="store_true", help="structured JSON log lines (KAFKA_LOG_JSON=1)")
    for flag, env in FLAGS.items():
        ap.add_argument("--" + flag.replace("_", "-"), default=None, help=f"overrides {env}")
    ap.add_argument("--ignore-eos", action="store_true", help="KAFKA_IGNORE_EOS=1 (benchmarks)")
    ap.add_argument("--mcp", action="store_true", help="KAFKA_MCP=1")
    a = ap.parse_args()
    for flag, env in FLAGS.items():
        v = getattr(a, flag)
        if v is not None:
            os.environ[env] = str(v)
    if a.ignore_eos:
        os.environ["KAFKA_IGNORE_EOS"] = "1"
    if a.mcp:
        os.environ["KAFKA_MCP"] = "1"
    if a.log_json:
        os.environ["KAFKA_LOG_JSON"] = "1"
    import uvicorn

    from kafka_llm_service_amd.obs.logging import setup_logging
    from kafka_llm_service_amd.server.app import create_app

    setup_logging()
    prof_path = os.environ.get("KAFKA_API_PROFILE")  # event-loop (main thread) profile, written at shutdown
    if not prof_path:
        uvicorn.run(create_app(), host=a.host, port=a.port, log_level=a.log_level, workers=1)
        return
    import cProfile
    import pstats

    import signal
    import sys

    # uvicorn re-raises the captured SIGTERM after its graceful shutdown: make that an exit that runs `finally`
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(0))
    prof = cProfile.Profile()
    try:
        prof.runcall(uvicorn.run, create_app(), host=a.host, port=a.port, log_level=a.log_level, workers=1)
    finally:
        with open(prof_path, "w") as f:
            st = pstats.Stats(prof, stream=f)
            st.sort_stats("tottime").print_stats(45)
            st.sort_stats("cumtime").print_stats(60)


if __name__ == "__main__":
    main()
