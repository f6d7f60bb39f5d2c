"""Utilities — mirror of the reference's ``src/utils`` (data_loader)."""
