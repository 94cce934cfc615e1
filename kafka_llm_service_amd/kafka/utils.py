"""Request-message helpers (/root/reference/src/kafka/utils.py:14-66)."""
from __future__ import annotations

import logging

from kafka_llm_service_amd.kafka.types import ChatMessage
from kafka_llm_service_amd.llm.types import Message

log = logging.getLogger("kafka")


def convert_to_internal_message(chat_msg: ChatMessage) -> Message:
    return Message(role=chat_msg.role, content=chat_msg.content, name=chat_msg.name, tool_calls=chat_msg.tool_calls,
                   tool_call_id=chat_msg.tool_call_id)


def sanitize_messages_for_openai(messages: list[Message]) -> list[Message]:
    """Drop tool messages that do not answer a tool call of the immediately preceding assistant turn.

    Only orphan tool messages are removed; every other message is kept untouched and in order, so the rendered
    history stays a token-prefix of the previous turn's (prefix-cache stability)."""
    out: list[Message] = []
    valid: set[str] = set()
    for m in messages:
        if m.role == "assistant" and m.tool_calls:
            valid = {tc.get("id") for tc in m.tool_calls if tc.get("id")}
            out.append(m)
        elif m.role == "tool":
            if m.tool_call_id and m.tool_call_id in valid:
                out.append(m)
                valid.discard(m.tool_call_id)
            else:
                log.warning("skipping orphan tool message (tool_call_id=%s, name=%s)", m.tool_call_id, m.name)
        else:
            valid = set()
            out.append(m)
    return out


def messages_to_dict_list(messages: list[Message]) -> list[dict]:
    return [m.to_dict() for m in messages]
