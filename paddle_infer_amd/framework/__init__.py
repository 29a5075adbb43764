"""Framework core: dtypes, places, RNG, parameter attributes, checkpoint IO, flags."""
