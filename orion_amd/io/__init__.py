"""File formats (YAML/JSON converters)."""
