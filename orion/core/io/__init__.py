"""``orion.core.io`` -> :mod:`orion_amd.io` / :mod:`orion_amd.store` / :mod:`orion_amd.space.dsl`."""
