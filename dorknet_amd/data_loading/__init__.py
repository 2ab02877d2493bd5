"""Device-side input pipeline (reference: data_loading/)."""
