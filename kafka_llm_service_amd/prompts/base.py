"""Section-based system-prompt composition with ``{{variable}}`` enrichment.

API parity with /root/reference/src/prompts/base.py:16-537 (PromptSection; PromptProvider with enrich /
clear_enrichment / get_section(_content) / list(_all)_sections / enable / disable / set_section_order / add_section /
remove_section / get_template_variables / get_missing_variables / get_system_prompt / validate). Unknown variables
are left verbatim. Rendering is deterministic (fixed section order, fixed separator), so the same provider state
always produces the same bytes — and therefore the same token prefix for the engine's prefix cache.
"""
from __future__ import annotations

import re
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any


@dataclass
class PromptSection:
    name: str
    content: str
    order: int = 0
    enabled: bool = True
    metadata: dict[str, Any] = field(default_factory=dict)

    def __post_init__(self):
        if not self.name:
            raise ValueError("Section name cannot be empty")
        if self.content is None:
            self.content = ""


class PromptProvider(ABC):
    TEMPLATE_PATTERN = re.compile(r"\{\{(\w+)\}\}")

    def __init__(self, enrichment: dict[str, Any] | None = None, sections: list[str] | None = None,
                 sections_dir: str | Path | None = None):
        self._enrichment_data: dict[str, Any] = dict(enrichment or {})
        self._sections_dir = Path(sections_dir) if sections_dir else None
        self._sections: dict[str, PromptSection] = {}
        self._section_order: list[str] = []
        self._requested = sections
        self._initialize_sections()

    def _initialize_sections(self) -> None:
        loaded = sorted(self._load_sections(), key=lambda s: s.order)
        for s in loaded:
            self._sections[s.name] = s
        names = [s.name for s in loaded]
        if self._requested is not None:
            for s in self._sections.values():
                s.enabled = s.name in self._requested
            names = [n for n in self._requested if n in self._sections] + \
                [n for n in names if n not in self._requested]
        self._section_order = names

    @abstractmethod
    def _load_sections(self) -> list[PromptSection]:
        ...

    @staticmethod
    def _load_section_from_file(path: Path, name: str, order: int) -> PromptSection | None:
        if not path.exists():
            return None
        return PromptSection(name=name, content=path.read_text(encoding="utf-8"), order=order,
                             metadata={"file": str(path)})

    def _load_sections_from_directory(self, directory: Path, start_order: int = 0) -> list[PromptSection]:
        out = []
        for i, p in enumerate(sorted(directory.glob("*.md"))):
            name = re.sub(r"^\d+_", "", p.stem)
            out.append(PromptSection(name=name, content=p.read_text(encoding="utf-8"),
                                     order=start_order + i, metadata={"file": str(p)}))
        return out

    # --- enrichment -------------------------------------------------------------------------------------------
    def enrich(self, data: dict[str, Any]) -> "PromptProvider":
        self._enrichment_data.update(data)
        return self

    def clear_enrichment(self) -> "PromptProvider":
        self._enrichment_data.clear()
        return self

    @property
    def enrichment(self) -> dict[str, Any]:
        return dict(self._enrichment_data)

    def _substitute_variables(self, content: str) -> str:
        def rep(m: re.Match) -> str:
            k = m.group(1)
            return str(self._enrichment_data[k]) if k in self._enrichment_data else m.group(0)

        return self.TEMPLATE_PATTERN.sub(rep, content)

    # --- sections ---------------------------------------------------------------------------------------------
    def get_section(self, name: str) -> PromptSection | None:
        return self._sections.get(name)

    def get_section_content(self, name: str, enrich: bool = True) -> str | None:
        s = self._sections.get(name)
        if s is None:
            return None
        return self._substitute_variables(s.content) if enrich else s.content

    def list_sections(self) -> list[str]:
        return [n for n in self._section_order if n in self._sections and self._sections[n].enabled]

    def list_all_sections(self) -> list[str]:
        return [n for n in self._section_order if n in self._sections]

    def enable_section(self, name: str) -> "PromptProvider":
        if name in self._sections:
            self._sections[name].enabled = True
        return self

    def disable_section(self, name: str) -> "PromptProvider":
        if name in self._sections:
            self._sections[name].enabled = False
        return self

    def set_section_order(self, order: list[str]) -> "PromptProvider":
        self._section_order = [n for n in order if n in self._sections] + \
            [n for n in self._section_order if n not in order]
        return self

    def add_section(self, name: str, content: str, order: int | None = None,
                    position: int | None = None) -> "PromptProvider":
        if order is None:
            order = max((s.order for s in self._sections.values()), default=0) + 1
        self._sections[name] = PromptSection(name=name, content=content, order=order)
        if name not in self._section_order:
            if position is not None:
                self._section_order.insert(position, name)
            else:
                # keep the list sorted by order so tail sections (custom instructions 999, playbooks 1000) land last
                idx = len(self._section_order)
                for i, n in enumerate(self._section_order):
                    if self._sections[n].order > order:
                        idx = i
                        break
                self._section_order.insert(idx, name)
        return self

    def remove_section(self, name: str) -> "PromptProvider":
        self._sections.pop(name, None)
        if name in self._section_order:
            self._section_order.remove(name)
        return self

    def get_template_variables(self) -> list[str]:
        seen: list[str] = []
        for n in self.list_sections():
            for v in self.TEMPLATE_PATTERN.findall(self._sections[n].content):
                if v not in seen:
                    seen.append(v)
        return seen

    def get_missing_variables(self) -> list[str]:
        return [v for v in self.get_template_variables() if v not in self._enrichment_data]

    def get_system_prompt(self, include_disabled: bool = False, separator: str = "\n\n") -> str:
        parts = []
        for n in self._section_order:
            s = self._sections.get(n)
            if s is None or (not s.enabled and not include_disabled):
                continue
            c = self._substitute_variables(s.content)
            if c.strip():
                parts.append(c)
        return separator.join(parts)

    def validate(self) -> dict[str, Any]:
        missing = self.get_missing_variables()
        empty = [n for n in self.list_sections() if not self._sections[n].content.strip()]
        return {"valid": not missing and not empty, "missing_variables": missing, "empty_sections": empty,
                "enabled_sections": self.list_sections(), "total_chars": len(self.get_system_prompt())}

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}(sections={self.list_sections()})"

    def __str__(self) -> str:
        return self.get_system_prompt()
