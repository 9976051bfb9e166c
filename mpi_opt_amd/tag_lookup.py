"""Message tags of the coordinator <-> block protocol (/root/reference/tag_lookup.py:1-12)."""

_TAGS = {"json": 1, "result": 2, "mbuilder": 3, "params": 4}


def tag_lookup(tag):
    """Integer of a tag name; 0 for unknown names."""
    return _TAGS.get(tag, 0)
