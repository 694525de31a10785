"""minips_amd subpackage."""
