"""Release / test tooling (the reference's py/ directory, re-targeted at a generic cluster)."""
