"""Interconnect tools: the standalone Booksim mode of the router model."""
