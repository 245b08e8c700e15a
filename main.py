"""FastTalk LLM service CLI (reference ``main.py``): modes ``websocket`` |
``config`` | ``test``; ``--provider`` adds ``native`` (in-process MI355X engine,
the default)."""
from __future__ import annotations

import argparse
import asyncio
import logging
import sys

from app.utils.config import Config
from app.utils.logger import get_logger

logging.basicConfig(level=logging.WARNING, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s",
                    stream=sys.stdout)
logger = get_logger(__name__)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="FastTalk LLM Service (MI355X)")
    p.add_argument("mode", choices=["websocket", "config", "test"], help="Operating mode")
    p.add_argument("--port", type=int, help="Server port")
    p.add_argument("--host", type=str, help="Server host")
    p.add_argument("--model", type=str, help="Model name / alias / checkpoint dir")
    p.add_argument("--provider", type=str, choices=["native", "vllm", "ollama", "openai"],
                   help="LLM provider")
    p.add_argument("--log-level", type=str, help="Logging level")
    p.add_argument("--show", action="store_true", help="Show configuration")
    return p


def apply_overrides(config: Config, args) -> Config:
    if args.port:
        config.port = args.port
    if args.host:
        config.host = args.host
    if args.provider:
        config.llm_provider = args.provider
    if args.model:
        if config.llm_provider in ("vllm", "openai"):
            config.vllm_model = args.model
        elif config.llm_provider == "native":
            config.engine_model = args.model
        else:
            config.model_name = args.model
    if args.log_level:
        config.log_level = args.log_level
        logging.getLogger().setLevel(args.log_level.upper())
    return config


def _test_connection(config: Config) -> int:
    print(f"\nTest mode - checking {config.llm_provider.upper()} backend...")
    print("=" * 50)
    if config.llm_provider == "native":
        from app.core.native_handler import NativeHandler

        h = NativeHandler(config)
        ok = h.check_connection()
        print(f"{'OK' if ok else 'FAIL'} native engine: {h.get_model_info()['engine']}")
        if ok:
            async def once():
                parts = []
                async for t in h.generate_stream_async([{"role": "user", "content": "Say hello."}],
                                                       temperature=0.0, max_tokens=8):
                    parts.append(t)
                return "".join(parts)

            print(f"OK sample generation: {asyncio.run(once())!r}")
        return 0 if ok else 1
    if config.llm_provider in ("vllm", "openai"):
        from app.core.vllm_handler import VLLMHandler

        ok = VLLMHandler(config.vllm_base_url, config.vllm_model, config.vllm_api_key).check_connection()
    else:
        from app.core.ollama_handler import OllamaHandler

        ok = OllamaHandler(config.ollama_base_url, config.model_name).check_connection()
    print(("OK" if ok else "FAIL") + f" {config.llm_provider} backend")
    return 0 if ok else 1


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    config = apply_overrides(Config(), args)
    if args.mode == "config":
        if args.show:
            print("\n" + "=" * 60 + "\nLLM Service Configuration\n" + "=" * 60)
            for k, v in config.to_dict().items():
                print(f"{k:30s}: {v}")
            print("=" * 60)
        return 0
    if args.mode == "test":
        return _test_connection(config)
    from app.core.websocket_launcher import WebSocketLauncher
    from app.monitoring.service_monitor import MonitoringServer

    monitoring = MonitoringServer(host=config.monitoring_host, port=config.monitoring_port)
    monitoring.start()
    WebSocketLauncher(config, monitor=monitoring.monitor).start()
    return 0


if __name__ == "__main__":
    sys.exit(main())
