"""Task launchers (reference: ``harness/determined/launch``)."""
