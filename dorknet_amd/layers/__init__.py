"""Layer classes: the reference's `layers` package (Layer protocol + concrete layers)."""
