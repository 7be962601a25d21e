# variant: the shipped sources unchanged (the variant differs only in its compiler flags)
