"""PromptProviderV1: the Kafka agent's default system prompt (13 sections: 7 core + 6 tool guides).

Structure parity with /root/reference/src/prompts/v1.py:15-298 (section names and order, default enrichment keys,
``create_minimal`` / ``create_tools_only`` / ``without_tools`` and the module factories).

Section text — two sets, picked by ``KAFKA_PROMPT`` (or the ``variant`` argument):
  * ``reference`` (default): ``prompts/sections_reference`` holds the reference's 13 section files verbatim, as DATA
    (SURVEY.md §2.1 #18 "copy as data"): the served prompt renders byte-identically to the reference's
    PromptProviderV1 with its default enrichment (/root/reference/src/prompts/v1.py:73-117) — 70,496 chars,
    ~16-17k Llama-3 tokens, the shared prefix every thread carries;
  * ``compact``: ``prompts/sections`` is this repo's own shorter wording of the same sections (47k chars).
The synthetic benchmark prefix in bench.py reproduces the reference prompt's token count either way.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any

from kafka_llm_service_amd.prompts.base import PromptProvider, PromptSection

SECTIONS_DIR = Path(__file__).resolve().parent / "sections"
REFERENCE_SECTIONS_DIR = Path(__file__).resolve().parent / "sections_reference"
PROMPT_VARIANTS = {"reference": REFERENCE_SECTIONS_DIR, "compact": SECTIONS_DIR}


def default_sections_dir(variant: str | None = None) -> Path:
    """Section directory of a prompt variant (``KAFKA_PROMPT`` when not given; default ``reference``)."""
    import os

    v = variant or os.environ.get("KAFKA_PROMPT", "reference")
    if v not in PROMPT_VARIANTS:
        raise ValueError(f"KAFKA_PROMPT must be one of {sorted(PROMPT_VARIANTS)}, got {v!r}")
    return PROMPT_VARIANTS[v]


class PromptProviderV1(PromptProvider):
    DEFAULT_ENRICHMENT: dict[str, Any] = {
        "working_language": "English", "sandbox_os": "Ubuntu 22.04", "sandbox_arch": "linux/amd64",
        "sandbox_user": "ubuntu", "sandbox_home": "/home/user", "sandbox_working_dir": "/workspace",
        "uploads_dir": "uploads/", "python_version": "3.10.12", "node_version": "20.18.0",
    }
    SECTION_FILES: dict[str, tuple] = {
        "intro": ("01_intro.md", None, 1), "core_principles": ("02_core_principles.md", None, 2),
        "core_tools": ("03_core_tools.md", None, 3), "decision_tree": ("04_decision_tree.md", None, 4),
        "workflow": ("05_workflow.md", None, 5), "environment": ("06_environment.md", None, 6),
        "operational": ("07_operational.md", None, 7), "notebook_shell": ("01_notebook_shell.md", "tools", 8),
        "search": ("02_search.md", "tools", 9), "webcrawler": ("03_webcrawler.md", "tools", 10),
        "agent": ("04_agent.md", "tools", 11), "domain_specific": ("05_domain_specific.md", "tools", 12),
        "appfactory": ("06_appfactory.md", "tools", 13),
    }
    DEFAULT_SECTION_ORDER = list(SECTION_FILES)
    TOOL_SECTIONS = ["notebook_shell", "search", "webcrawler", "agent", "domain_specific", "appfactory"]

    def __init__(self, enrichment: dict[str, Any] | None = None, sections: list[str] | None = None,
                 sections_dir: str | Path | None = None, use_defaults: bool = True, variant: str | None = None):
        data = dict(self.DEFAULT_ENRICHMENT) if use_defaults else {}
        data.update(enrichment or {})
        self.variant = variant
        super().__init__(enrichment=data, sections=sections,
                         sections_dir=sections_dir or default_sections_dir(variant))

    def _load_sections(self) -> list[PromptSection]:
        out = []
        for name, (fname, sub, order) in self.SECTION_FILES.items():
            path = self._sections_dir / sub / fname if sub else self._sections_dir / fname
            s = self._load_section_from_file(path, name, order)
            if s is not None:
                out.append(s)
        return out

    @classmethod
    def get_default_enrichment(cls) -> dict[str, Any]:
        return dict(cls.DEFAULT_ENRICHMENT)

    @classmethod
    def get_available_sections(cls) -> list[str]:
        return list(cls.SECTION_FILES)

    def create_minimal(self) -> "PromptProviderV1":
        return PromptProviderV1(enrichment=self.enrichment, sections=["intro", "core_principles", "workflow"],
                                sections_dir=self._sections_dir, use_defaults=False)

    def create_tools_only(self) -> "PromptProviderV1":
        return PromptProviderV1(enrichment=self.enrichment, sections=list(self.TOOL_SECTIONS),
                                sections_dir=self._sections_dir, use_defaults=False)

    def without_tools(self) -> "PromptProviderV1":
        return PromptProviderV1(enrichment=self.enrichment,
                                sections=[s for s in self.DEFAULT_SECTION_ORDER if s not in self.TOOL_SECTIONS],
                                sections_dir=self._sections_dir, use_defaults=False)


def create_default_provider(**enrichment) -> PromptProviderV1:
    return PromptProviderV1(enrichment=enrichment)


def create_minimal_provider(**enrichment) -> PromptProviderV1:
    return PromptProviderV1(enrichment=enrichment, sections=["intro", "core_principles", "workflow"])


def create_custom_provider(sections: list[str], **enrichment) -> PromptProviderV1:
    return PromptProviderV1(enrichment=enrichment, sections=sections)
