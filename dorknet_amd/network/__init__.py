"""Network container (the reference's `network` package)."""
