"""Placeholder module for the larger zoo members (registered on import)."""
