"""``get_weather``: Open-Meteo geocoding + current conditions (/root/reference/server_tools/weather.py:13-112).

The build/GPU hosts have no network, so ``KAFKA_WEATHER_MODE=offline`` (the default when the API is unreachable)
answers from a deterministic fixture table; ``online`` forces the HTTP path.
"""
from __future__ import annotations

import hashlib
import os

from kafka_llm_service_amd.tools.types import Tool

WEATHER_CODES = {0: "Clear sky", 1: "Mainly clear", 2: "Partly cloudy", 3: "Overcast", 45: "Foggy",
                 48: "Depositing rime fog", 51: "Light drizzle", 53: "Moderate drizzle", 55: "Dense drizzle",
                 61: "Slight rain", 63: "Moderate rain", 65: "Heavy rain", 71: "Slight snow", 73: "Moderate snow",
                 75: "Heavy snow", 80: "Slight rain showers", 81: "Moderate rain showers",
                 82: "Violent rain showers", 95: "Thunderstorm", 96: "Thunderstorm with slight hail",
                 99: "Thunderstorm with heavy hail"}

FIXTURES = {"new york": ("New York", "United States"), "london": ("London", "United Kingdom"),
            "paris": ("Paris", "France"), "tokyo": ("Tokyo", "Japan"), "san francisco": ("San Francisco",
                                                                                          "United States"),
            "berlin": ("Berlin", "Germany"), "istanbul": ("Istanbul", "Turkey")}


def _format(name, country, code, temp, feels, hum, wind, precip, unit):
    sym = "°F" if unit == "fahrenheit" else "°C"
    return (f"Weather in {name}, {country}:\n• Condition: {WEATHER_CODES.get(code, 'Unknown')}\n"
            f"• Temperature: {temp}{sym} (feels like {feels}{sym})\n• Humidity: {hum}%\n• Wind: {wind} mph\n"
            f"• Precipitation: {precip} mm")


def offline_weather(location: str, units: str = "celsius") -> str:
    key = location.lower().split(",")[0].strip()
    if key not in FIXTURES and not key:
        return f"Could not find location: {location}"
    name, country = FIXTURES.get(key, (location.split(",")[0].strip().title(), "Unknown"))
    h = int(hashlib.sha1(key.encode()).hexdigest(), 16)
    code = sorted(WEATHER_CODES)[h % len(WEATHER_CODES)]
    c = round(-5 + (h % 3500) / 100.0, 1)
    unit = "fahrenheit" if units.lower() == "fahrenheit" else "celsius"
    t = round(c * 9 / 5 + 32, 1) if unit == "fahrenheit" else c
    return _format(name, country, code, t, round(t - 1.5, 1), 30 + h % 60, round((h % 250) / 10, 1),
                   round((h % 50) / 10, 1), unit)


async def get_weather(location: str, units: str = "celsius") -> str:
    mode = os.environ.get("KAFKA_WEATHER_MODE", "auto")
    if mode == "offline":
        return offline_weather(location, units)
    import httpx

    try:
        async with httpx.AsyncClient(timeout=10.0) as client:
            g = (await client.get("https://geocoding-api.open-meteo.com/v1/search",
                                  params={"name": location, "count": 1, "language": "en", "format": "json"})).json()
            if not g.get("results"):
                return f"Could not find location: {location}"
            r = g["results"][0]
            unit = "fahrenheit" if units.lower() == "fahrenheit" else "celsius"
            w = (await client.get("https://api.open-meteo.com/v1/forecast", params={
                "latitude": r["latitude"], "longitude": r["longitude"],
                "current": "temperature_2m,relative_humidity_2m,apparent_temperature,precipitation,weather_code,"
                           "wind_speed_10m", "temperature_unit": unit, "wind_speed_unit": "mph",
                "timezone": "auto"})).json().get("current", {})
            return _format(r.get("name", location), r.get("country", ""), w.get("weather_code", 0),
                           w.get("temperature_2m", "N/A"), w.get("apparent_temperature", "N/A"),
                           w.get("relative_humidity_2m", "N/A"), w.get("wind_speed_10m", "N/A"),
                           w.get("precipitation", 0), unit)
    except (httpx.HTTPError, ValueError, KeyError):
        if mode == "online":
            raise
        return offline_weather(location, units)


get_weather_tool = Tool(
    name="get_weather",
    description="Get the current weather for a location. Returns temperature, conditions, humidity, and wind speed.",
    parameters={"type": "object", "properties": {
        "location": {"type": "string", "description": "City name or location, e.g. 'New York' or 'London, UK'"},
        "units": {"type": "string", "enum": ["celsius", "fahrenheit"], "description": "Temperature units",
                  "default": "celsius"}}, "required": ["location"]},
    handler=get_weather)
