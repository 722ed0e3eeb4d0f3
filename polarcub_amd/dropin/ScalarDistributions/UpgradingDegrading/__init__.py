"""Drop-in package (see polarcub_amd/dropin/README.md)."""
