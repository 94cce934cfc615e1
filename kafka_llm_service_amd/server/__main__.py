"""``python -m kafka_llm_service_amd.server`` — run the API server (the reference's ``python server.py``, port 8081 by
default, /root/reference/server.py:627-631). Configuration comes from the environment (``ServerConfig.from_env``:
KAFKA_LLM_BACKEND, KAFKA_MODEL, KAFKA_DP, KAFKA_TP, LOCAL_DB_PATH, KAFKA_SANDBOX, LOCAL_SANDBOX_URL, ...)."""
from __future__ import annotations

import argparse
import os


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default=os.environ.get("HOST", "0.0.0.0"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("PORT", "8081")))
    ap.add_argument("--log-level", default="warning")
    a = ap.parse_args()
    import uvicorn

    from kafka_llm_service_amd.server.app import create_app

    uvicorn.run(create_app(), host=a.host, port=a.port, log_level=a.log_level, workers=1)


if __name__ == "__main__":
    main()
